// lab_lookback.h -- LAB ONLY (tools/lab, libmcodec_lab.so; never in
// libmcodec.so): decoupled look-back primitives of the single-pass scan
// schedules that DESIGN.md measured against the product's 3-pass scans.
#pragma once

#include "mc_scan.h"

// (lab) single-pass scan across workgroups (decoupled look-back) for the
// one-launch Delta / FSO->Delta->Shuffle decodes (lab_scan1p.hip).
//
// Partitions are numbered by an atomic ticket in workgroup START order
// (mc_lb_ticket), so every predecessor a partition waits on belongs to a
// workgroup that is already running: progress never depends on dispatch
// order or on how many workgroups are resident.  Each partition publishes
// one 64-bit status word {flag:32 | value:32} -- first its aggregate (flag
// 1), then its inclusive prefix (flag 2) -- with ONE agent-scope relaxed
// 64-bit atomic store, read with agent-scope relaxed atomic loads: the value
// travels with its flag in one granule, so no release/acquire fence is needed
// (MI355X_MICROARCH.md, "R2" granule hand-off).  Values are kept mod 2^32,
// exact for every accumulation width <= 32 bits.
//
// Workspace: [0] ticket counter, [1] retire counter, [2] fallback count,
// [3] pad, then one status word per partition.  It must be zero before the
// first launch; the last workgroup to retire zeroes it again (mc_lb_retire),
// so a launch leaves it ready for the next launch on the same stream.

typedef __attribute__((address_space(1))) uint64_t mc_gu64;
typedef __attribute__((address_space(1))) uint32_t mc_gu32;

constexpr uint64_t MC_LB_AGG = 1ull << 32;
constexpr uint64_t MC_LB_INC = 2ull << 32;
// Spin bound of a look-back round (s_sleep(1) between polls).  With ticket
// order a predecessor is always running, so the bound is only a guard: a
// partition that hits it derives its prefix from the data itself (correct,
// slow) and counts it in workspace word [2].
constexpr unsigned MC_LB_WAVE_SPINS = 1u << 14;

static inline size_t mc_lb_ws_bytes(size_t npart) { return 16 + 8 * npart; }

// Whole block: the next partition ticket (thread 0's atomicAdd, broadcast
// through `slot`).
MC_DEV size_t mc_lb_ticket(uint32_t *counter, uint32_t *slot) {
  if (threadIdx.x == 0) *slot = atomicAdd(counter, 1u);
  __syncthreads();
  const size_t t = *slot;
  __syncthreads();
  return t;
}

MC_DEV void mc_lb_publish_aggregate(uint64_t *status_, size_t tile, uint32_t aggregate) {
  __hip_atomic_store(&((mc_gu64 *)status_)[tile], MC_LB_AGG | aggregate, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

MC_DEV void mc_lb_publish_inclusive(uint64_t *status_, size_t tile, uint32_t inclusive) {
  __hip_atomic_store(&((mc_gu64 *)status_)[tile], MC_LB_INC | inclusive, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}


// ---------------------------------------------------------------------------
// Block-wide look-back: the 256 threads read 4 status words each, a window of
// the 1024 partitions below `base` per round (one round reaches back over a
// whole generation of resident workgroups).  The caller issues the first
// round's loads itself (mc_lb_block_poll) BEFORE its streaming loads, so that
// waiting for the status words does not wait for those loads (vmcnt retires
// in issue order; the compiler waits only for what a use needs).
// ---------------------------------------------------------------------------
struct McLbBlock {
  uint32_t first[MC_BLOCK / 64];
  uint32_t sum[MC_BLOCK / 64];
};

MC_DEV void mc_lb_block_poll(const uint64_t *status_, long long base, uint64_t (&s)[4]) {
  mc_gu64 *status = (mc_gu64 *)status_;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long idx = base - 4 * (long long)threadIdx.x - q;
    s[q] = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : MC_LB_INC;  // before partition 0: an inclusive prefix of 0
  }
}

// block-wide minimum of one value per thread (two __syncthreads)
MC_DEV uint32_t mc_block_min(uint32_t v, uint32_t *red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t m = red[0];
#pragma unroll
  for (int w = 1; w < MC_BLOCK / 64; ++w) m = red[w] < m ? red[w] : m;
  __syncthreads();
  return m;
}

// Every thread of the block: the exclusive prefix of `tile` (aggregate
// already published) from the first round's words `s` (polled at
// base = tile - 1); publishes the inclusive prefix.
//
// Window position g = 4 * thread + slot counts back from `base` (g = 0 is
// the nearest predecessor).  Only the run of words nearer than the nearest
// inclusive prefix matters: if the nearest non-aggregate word is an
// inclusive prefix the walk ends there; if it is an unpublished word, the
// aggregates before it are banked, the window moves to start at it and is
// re-polled after a short sleep (words beyond it are never waited for); a
// window of aggregates only is banked whole and the walk moves 1024 back.
// After `max_spins` re-polls `ok` is false (block-uniform) and nothing is
// published -- the caller then derives the prefix from the data.
MC_DEV uint32_t mc_lb_block_lookback(uint64_t *status_, size_t tile, uint32_t aggregate, uint64_t (&s)[4],
                                     unsigned max_spins, bool &ok, McLbBlock &sh) {
  constexpr uint32_t NONE = 0xffffffffu;
  long long base = (long long)tile - 1;
  uint32_t prefix = 0;
  unsigned spins = 0;
  ok = true;
  for (;;) {
    uint32_t my_inc = NONE, my_pend = NONE;
#pragma unroll
    for (int q = 3; q >= 0; --q) {  // nearest slot last, so it wins
      const uint32_t flag = (uint32_t)(s[q] >> 32);
      const uint32_t g = 4 * threadIdx.x + q;
      if (flag == 2) my_inc = g;
      if (flag == 0) my_pend = g;
    }
    const uint32_t g_inc = mc_block_min(my_inc, sh.first);
    const uint32_t g_pend = mc_block_min(my_pend, sh.first);
    const bool done = g_inc < g_pend;                  // an inclusive prefix before any gap
    const uint32_t lim = done ? g_inc + 1 : (g_pend == NONE ? 4 * MC_BLOCK : g_pend);
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * threadIdx.x + q < lim) v += (uint32_t)s[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) sh.sum[threadIdx.x >> 6] = v;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < MC_BLOCK / 64; ++w) prefix += sh.sum[w];
    __syncthreads();  // sh is rewritten by the next round
    if (done) break;
    base -= lim;  // banked: the words before the gap (or the whole window)
    if (g_pend != NONE) {
      if (++spins > max_spins) {
        ok = false;
        return 0;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    mc_lb_block_poll(status_, base, s);
  }
  if (threadIdx.x == 0) mc_lb_publish_inclusive(status_, tile, prefix + aggregate);
  return prefix;
}

// Whole block, once, after its last ticket: the last workgroup to retire
// (every other one has finished all its status reads) zeroes the ticket
// counter, the retire counter and the status words for the next launch.
MC_DEV void mc_lb_retire(uint32_t *ws, size_t npart, uint32_t *slot) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(&ws[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    *slot = old == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (*slot) {
    uint64_t *status = reinterpret_cast<uint64_t *>(ws + 4);
    for (size_t i = threadIdx.x; i < npart; i += blockDim.x) status[i] = 0;
    if (threadIdx.x == 0) {
      ws[0] = 0;
      ws[1] = 0;
    }
  }
}

// Exclusive block scans of R per-thread values at once, mod 2^32: one wave
// scan per value and ONE LDS round; excl[r] = this thread's exclusive prefix
// of value r, tot[r] = the block total of value r.  Two __syncthreads.
template <int R>
MC_DEV void mc_block_excl_scan_multi(const uint32_t (&x)[R], uint32_t (&excl)[R], uint32_t (&tot)[R],
                                     uint32_t (*red)[MC_BLOCK / 64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    incl[r] = x[r];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(incl[r], off, 64);
      if (lane >= off) incl[r] += o;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int r = 0; r < R; ++r) red[r][wave] = incl[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint32_t wpre = 0, t = 0;
#pragma unroll
    for (int w = 0; w < MC_BLOCK / 64; ++w) {
      const uint32_t val = red[r][w];
      if (w < wave) wpre += val;
      t += val;
    }
    excl[r] = wpre + incl[r] - x[r];
    tot[r] = t;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Decoupled look-back (single-pass scan across workgroups).
//
// Tiles are numbered in workgroup START order by an atomic counter, so the
// tile a workgroup waits on has always been started already (no dependence
// on dispatch order or residency).  Each tile publishes one 64-bit status
// word {flag:32 | value:32}: first its aggregate (flag 1), then its
// inclusive prefix (flag 2).  A word is written and read with ONE agent-scope
// relaxed 64-bit atomic (global_store/load_dwordx2 sc1): the value travels
// with its flag in the same granule, so no release/acquire fence is needed
// (MI355X_MICROARCH.md, "R2" granule hand-off).  Values are kept mod 2^32,
// exact for every accumulation width <= 32 bits.  Every spin is bounded: on
// timeout the tile sets *error and continues with what it has (the host turns
// that into an error).  The counter and the status words are zeroed by a
// hipMemsetAsync on the stream before every launch.
// ---------------------------------------------------------------------------
constexpr unsigned MC_LB_SPIN_LIMIT = 1u << 22;

// thread 0 of a block: the block's tile index (broadcast through `slot`)
MC_DEV size_t mc_lb_tile(uint32_t *counter, uint32_t *slot) {
  if (threadIdx.x == 0) *slot = atomicAdd(counter, 1u);
  __syncthreads();
  const size_t t = *slot;
  __syncthreads();
  return t;
}

// Called by ONE thread: publish `aggregate` for `tile`, look back for the
// exclusive prefix, publish the inclusive prefix; returns the exclusive prefix.
template <bool OR_OP>
MC_DEV uint32_t mc_lb_lookback(uint64_t *status_, size_t tile, uint32_t aggregate,
                               uint32_t *error) {
  mc_gu64 *status = (mc_gu64 *)status_;
  if (tile == 0) {
    __hip_atomic_store(&status[0], MC_LB_INC | aggregate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  __hip_atomic_store(&status[tile], MC_LB_AGG | aggregate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t prefix = 0;
  size_t j = tile - 1;
  unsigned spins = 0;
  for (;;) {
    const uint64_t s = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t flag = (uint32_t)(s >> 32);
    if (flag == 0) {
      if (++spins > MC_LB_SPIN_LIMIT) {
        __hip_atomic_store((mc_gu32 *)error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    prefix = OR_OP ? (prefix | (uint32_t)s) : (prefix + (uint32_t)s);
    if (flag == 2 || j == 0) break;
    --j;
  }
  const uint32_t inc = OR_OP ? (prefix | aggregate) : (prefix + aggregate);
  __hip_atomic_store(&status[tile], MC_LB_INC | inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return prefix;
}

// Wave-parallel variant, called by ALL 64 lanes of ONE wave: each round reads
// the status of 64 predecessors at once, so the walk back to the nearest
// inclusive prefix takes distance/64 dependent round trips.  Returns the
// exclusive prefix in every lane and publishes the tile's inclusive prefix.
// If a predecessor stays unpublished for MC_LB_WAVE_SPINS rounds, `ok` is set
// false (wave-uniform) and nothing more is published: the caller then derives
// the prefix from the data itself and publishes it (always correct, whatever
// the dispatch order).

template <bool OR_OP>
MC_DEV uint32_t mc_lb_lookback_wave(uint64_t *status_, size_t tile, uint32_t aggregate, bool &ok,
                                    unsigned max_spins = MC_LB_WAVE_SPINS) {
  mc_gu64 *status = (mc_gu64 *)status_;
  const int lane = threadIdx.x & 63;
  ok = true;
  if (tile == 0) {
    if (lane == 0)
      __hip_atomic_store(&status[0], MC_LB_INC | aggregate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(&status[tile], MC_LB_AGG | aggregate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t prefix = 0;
  long long base = (long long)tile - 1;  // predecessor read by lane 0
  unsigned spins = 0;
  for (;;) {
    const long long idx = base - lane;
    uint64_t s = MC_LB_INC;  // before tile 0: an inclusive prefix of 0
    if (idx >= 0) s = __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t flag = (uint32_t)(s >> 32);
    if (__any(flag == 0)) {
      if (++spins > max_spins) {
        ok = false;
        return 0;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const unsigned long long inc = __ballot(flag == 2);
    const int first = inc ? __ffsll((long long)inc) - 1 : 63;  // nearest inclusive prefix
    uint32_t v = lane <= first ? (uint32_t)s : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t o = __shfl_xor(v, off, 64);
      v = OR_OP ? (v | o) : (v + o);
    }
    prefix = OR_OP ? (prefix | v) : (prefix + v);
    if (inc) break;
    base -= 64;
  }
  if (lane == 0) {
    const uint32_t incv = OR_OP ? (prefix | aggregate) : (prefix + aggregate);
    __hip_atomic_store(&status[tile], MC_LB_INC | incv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return prefix;
}

// workspace layout for a look-back scan over ntiles tiles:
//   [0, 16): counter (u32) + error word (u32) + pad;  [16, 16 + 8*ntiles): status
static inline size_t mc_lb_workspace(size_t ntiles) { return 16 + 8 * ntiles; }

// Wider variant for coarse partitions: every lane reads 4 consecutive
// predecessors per round (256 per round, the 4 loads in flight together), so
// the walk back to the nearest inclusive prefix takes distance/256 round
// trips.  Same contract as mc_lb_lookback_wave.
template <bool OR_OP>
MC_DEV uint32_t mc_lb_lookback_wave4(uint64_t *status_, size_t tile, uint32_t aggregate, bool &ok,
                                     unsigned max_spins = MC_LB_WAVE_SPINS) {
  // window position g = 4 * lane + slot counts back from `base`; only the
  // words nearer than the nearest inclusive prefix are waited for (round-2
  // fix: the round-1 version waited for every word of the 256-window)
  mc_gu64 *status = (mc_gu64 *)status_;
  const int lane = threadIdx.x & 63;
  ok = true;
  if (tile == 0) {
    if (lane == 0)
      __hip_atomic_store(&status[0], MC_LB_INC | aggregate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0)
    __hip_atomic_store(&status[tile], MC_LB_AGG | aggregate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t prefix = 0;
  long long base = (long long)tile - 1;  // nearest predecessor: lane 0, slot 0
  unsigned spins = 0;
  for (;;) {
    uint64_t s[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long idx = base - 4 * lane - q;
      s[q] = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : MC_LB_INC;  // before tile 0: an inclusive prefix of 0
    }
    int my_inc = 1 << 30, my_pend = 1 << 30;
#pragma unroll
    for (int q = 3; q >= 0; --q) {
      const uint32_t flag = (uint32_t)(s[q] >> 32);
      if (flag == 2) my_inc = 4 * lane + q;
      if (flag == 0) my_pend = 4 * lane + q;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const int a = __shfl_xor(my_inc, off, 64), b = __shfl_xor(my_pend, off, 64);
      my_inc = a < my_inc ? a : my_inc;
      my_pend = b < my_pend ? b : my_pend;
    }
    const bool done = my_inc < my_pend;
    const int lim = done ? my_inc + 1 : (my_pend == (1 << 30) ? 256 : my_pend);
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * lane + q < lim) v = OR_OP ? (v | (uint32_t)s[q]) : (v + (uint32_t)s[q]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t o = __shfl_xor(v, off, 64);
      v = OR_OP ? (v | o) : (v + o);
    }
    prefix = OR_OP ? (prefix | v) : (prefix + v);
    if (done) break;
    base -= lim;
    if (my_pend != (1 << 30)) {
      if (++spins > max_spins) {
        ok = false;
        return 0;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  if (lane == 0) {
    const uint32_t incv = OR_OP ? (prefix | aggregate) : (prefix + aggregate);
    __hip_atomic_store(&status[tile], MC_LB_INC | incv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return prefix;
}
