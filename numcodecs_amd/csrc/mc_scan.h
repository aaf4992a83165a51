// mc_scan.h -- block/wave scan building blocks shared by the Delta decode
// scan (mc_scan.hip) and the fused FSO->Delta->Shuffle decode (mc_c4.hip).
#pragma once

#include "mc_num.h"

constexpr int MC_SCAN_STEPS = 4;
constexpr int MC_SCAN_TILE = 4 * MC_SCAN_STEPS * MC_BLOCK;  // 4096 elements

template <bool OR_OP>
MC_DEV uint64_t mc_scan_combine(uint64_t a, uint64_t b) {
  if constexpr (OR_OP) return a | b;
  else return a + b;
}

template <bool OR_OP>
MC_DEV uint64_t mc_wave_incl_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t o = __shfl_up(v, off, 64);
    if (lane >= off) v = mc_scan_combine<OR_OP>(v, o);
  }
  return v;
}

// Exclusive scan across the blockDim.x (<= 1024) threads of a block: returns
// this thread's exclusive prefix; *total = block total.  `lds` holds
// blockDim.x/64 words.  Contains two __syncthreads().
template <bool OR_OP>
MC_DEV uint64_t mc_block_excl_scan(uint64_t v, uint64_t *lds, uint64_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = (blockDim.x + 63) >> 6;
  const uint64_t incl = mc_wave_incl_scan<OR_OP>(v);
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  uint64_t wpre = 0, tot = 0;
  for (int w = 0; w < nwaves; ++w) {
    const uint64_t x = lds[w];
    if (w < wave) wpre = mc_scan_combine<OR_OP>(wpre, x);
    tot = mc_scan_combine<OR_OP>(tot, x);
  }
  __syncthreads();
  *total = tot;
  const uint64_t excl_in_wave = __shfl_up(incl, 1, 64);
  return mc_scan_combine<OR_OP>(wpre, lane ? excl_in_wave : 0);
}

// 32-bit exclusive block sum scan (mod 2^32): half the shuffle traffic of the
// 64-bit mc_block_excl_scan for callers whose totals are 32-bit (the int16 /
// int32 C4 scan).  Same contract: two __syncthreads(), `lds` holds
// blockDim.x/64 words.
MC_DEV uint32_t mc_block_excl_scan32(uint32_t v, uint32_t *lds, uint32_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = (blockDim.x + 63) >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
  for (int w = 0; w < nwaves; ++w) {
    const uint32_t x = lds[w];
    if (w < wave) wpre += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  const uint32_t excl_in_wave = __shfl_up(incl, 1, 64);
  return wpre + (lane ? excl_in_wave : 0u);
}

// Exclusive scan of `ntiles` tile totals in place, one workgroup of 1024
// (tools/scan_bench.hip measures it alone).  Per round of 8192 totals each
// wave moves its 512 through an LDS slice with coalesced global accesses
// (lane l loads l + 64k) and scans them as 8 consecutive totals per lane
// (serial adds), so one block scan -- one wave scan per wave -- is all the
// cross-lane work.  Two layouts measured slower: 16 consecutive totals per
// lane straight from global (each load instruction touches 64 cache lines on
// one CU: 18.7 us for 16K totals), 64-lane columns scanned across the wave
// (16 wave scans of 64-bit shuffles per round: 15.5 us) and 16K-total rounds
// (a 128 KiB LDS workgroup adds ~4 us of fixed cost).  This one: 9.2 us for
// 16K totals, 4.8 us for one round, the next round's loads issued early.
template <bool OR_OP>
__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t *__restrict__ sums, size_t ntiles) {
  constexpr int PER = 8, WSPAN = 64 * PER, ROUND = 1024 * PER;  // 64 KiB LDS
  __shared__ uint64_t red[1024 / 64];
  __shared__ __attribute__((aligned(16))) uint64_t buf[ROUND];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t *wbuf = buf + wave * WSPAN;
  uint64_t carry = 0;
  const size_t last = ntiles - 1;
  uint64_t x[PER];  // this round's totals; the next round's are loaded early
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const size_t i = (size_t)wave * WSPAN + lane + 64 * k;
    x[k] = sums[i < last ? i : last];
  }
  for (size_t r0 = 0; r0 < ntiles; r0 += ROUND) {
    const size_t wb = r0 + (size_t)wave * WSPAN + lane;
    uint64_t xn[PER];
    if (r0 + ROUND < ntiles) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const size_t i = wb + ROUND + 64 * k;
        xn[k] = sums[i < last ? i : last];
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) wbuf[lane + 64 * k] = wb + 64 * k < ntiles ? x[k] : 0;
    // the wave reads back what it wrote: no barrier needed, only LDS ordering
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    uint64_t v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = wbuf[PER * lane + k];
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint64_t t = v[k];
      v[k] = run;
      run = mc_scan_combine<OR_OP>(run, t);
    }
    uint64_t tot;
    const uint64_t excl = mc_scan_combine<OR_OP>(carry, mc_block_excl_scan<OR_OP>(run, red, &tot));
#pragma unroll
    for (int k = 0; k < PER; ++k) wbuf[PER * lane + k] = mc_scan_combine<OR_OP>(excl, v[k]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (wb + 64 * k < ntiles) sums[wb + 64 * k] = wbuf[lane + 64 * k];
    carry = mc_scan_combine<OR_OP>(carry, tot);
    if (r0 + ROUND < ntiles) {
#pragma unroll
      for (int k = 0; k < PER; ++k) x[k] = xn[k];
    }
  }
}

template <bool OR_OP>
static inline void mc_launch_scan_sums(uint64_t *sums, size_t ntiles, hipStream_t st) {
  k_scan_sums<OR_OP><<<1, 1024, 0, st>>>(sums, ntiles);
}

// Exclusive scan of n totals into a separate array by one workgroup per 256
// totals: workgroup g combines every total before its range itself
// (coalesced, 8 loads in flight per thread) and scans its own 256.  The
// one-workgroup k_scan_sums is bound by a single CU (4.8 us for one round of
// 8192, ~8 us in the C4 decode); reading the earlier totals redundantly
// spreads the work over n/256 CUs.  Not in place (in != out).
template <bool OR_OP>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_sums_mw(const uint64_t *__restrict__ in,
                                                          uint64_t *__restrict__ out, size_t n) {
  __shared__ uint64_t red[MC_BLOCK / 64];
  __shared__ uint64_t base_lds[MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t b = (size_t)blockIdx.x * MC_BLOCK;
  uint64_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t i = threadIdx.x;
  for (; i + 7 * MC_BLOCK < b; i += 8 * MC_BLOCK) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = mc_scan_combine<OR_OP>(a[k], in[i + (size_t)k * MC_BLOCK]);
  }
  for (; i < b; i += MC_BLOCK) a[0] = mc_scan_combine<OR_OP>(a[0], in[i]);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc = mc_scan_combine<OR_OP>(acc, a[k]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc = mc_scan_combine<OR_OP>(acc, __shfl_xor(acc, off, 64));
  if (lane == 0) base_lds[wave] = acc;
  const uint64_t x = b + threadIdx.x < n ? in[b + threadIdx.x] : 0;
  uint64_t tot;
  const uint64_t ex = mc_block_excl_scan<OR_OP>(x, red, &tot);  // its barriers publish base_lds
  uint64_t base = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) base = mc_scan_combine<OR_OP>(base, base_lds[w]);
  if (b + threadIdx.x < n) out[b + threadIdx.x] = mc_scan_combine<OR_OP>(base, ex);
}

template <bool OR_OP>
static inline void mc_launch_scan_sums_mw(const uint64_t *in, uint64_t *out, size_t n, hipStream_t st) {
  k_scan_sums_mw<OR_OP><<<(unsigned)((n + MC_BLOCK - 1) / MC_BLOCK), MC_BLOCK, 0, st>>>(in, out, n);
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
typedef __attribute__((address_space(1))) uint64_t mc_gu64;
typedef __attribute__((address_space(1))) uint32_t mc_gu32;

constexpr uint64_t MC_LB_AGG = 1ull << 32;
constexpr uint64_t MC_LB_INC = 2ull << 32;
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
constexpr unsigned MC_LB_WAVE_SPINS = 1u << 14;

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

// workspace layout for a look-back scan over ntiles tiles:
//   [0, 16): counter (u32) + error word (u32) + pad;  [16, 16 + 8*ntiles): status
static inline size_t mc_lb_workspace(size_t ntiles) { return 16 + 8 * ntiles; }
