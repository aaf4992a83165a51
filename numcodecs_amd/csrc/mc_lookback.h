// mc_lookback.h -- single-pass scan across workgroups (decoupled look-back)
// for the one-launch Delta / FSO->Delta->Shuffle decodes (mc_scan1p.hip).
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
#pragma once

#include "mc_scan.h"

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

// Wider variant for coarse partitions: every lane reads 4 consecutive
// predecessors per round (256 per round, the 4 loads in flight together), so
// the walk back to the nearest inclusive prefix takes distance/256 round
// trips.  Same contract as mc_lb_lookback_wave.
template <bool OR_OP>
MC_DEV uint32_t mc_lb_lookback_wave4(uint64_t *status_, size_t tile, uint32_t aggregate, bool &ok,
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
    bool pending = false;
    int fq = 4;  // this lane's nearest inclusive slot
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t flag = (uint32_t)(s[q] >> 32);
      pending |= flag == 0;
      if (fq == 4 && flag == 2) fq = q;
    }
    if (__any(pending)) {
      if (++spins > max_spins) {
        ok = false;
        return 0;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const unsigned long long inc = __ballot(fq < 4);
    const int first = inc ? __ffsll((long long)inc) - 1 : 64;  // nearest lane holding an inclusive
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool take = lane < first || (lane == first && q <= fq);
      if (take) v = OR_OP ? (v | (uint32_t)s[q]) : (v + (uint32_t)s[q]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t o = __shfl_xor(v, off, 64);
      v = OR_OP ? (v | o) : (v + o);
    }
    prefix = OR_OP ? (prefix | v) : (prefix + v);
    if (inc) break;
    base -= 256;
  }
  if (lane == 0) {
    const uint32_t incv = OR_OP ? (prefix | aggregate) : (prefix + aggregate);
    __hip_atomic_store(&status[tile], MC_LB_INC | incv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return prefix;
}

MC_DEV void mc_lb_publish_inclusive(uint64_t *status_, size_t tile, uint32_t inclusive) {
  __hip_atomic_store(&((mc_gu64 *)status_)[tile], MC_LB_INC | inclusive, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
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
