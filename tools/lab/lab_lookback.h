// lab_lookback.h -- LAB ONLY (tools/lab, libmcodec_lab.so; never in
// libmcodec.so): decoupled look-back primitives of the single-pass scan
// schedules that DESIGN.md measured against the product's 3-pass scans.
#pragma once

#include "mc_lookback.h"

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
