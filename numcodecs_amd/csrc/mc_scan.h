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

// Exclusive scan of `ntiles` tile totals in place, one workgroup of 1024:
// rounds of 4096 totals staged through LDS with coalesced loads and stores.
template <bool OR_OP>
__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t *__restrict__ sums, size_t ntiles) {
  constexpr int PER = 4, ROUND = 1024 * PER;
  __shared__ uint64_t buf[ROUND];
  __shared__ uint64_t red[1024 / 64];
  uint64_t carry = 0;
  for (size_t r0 = 0; r0 < ntiles; r0 += ROUND) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const size_t i = r0 + (size_t)j * 1024 + threadIdx.x;
      buf[j * 1024 + threadIdx.x] = i < ntiles ? sums[i] : 0;
    }
    __syncthreads();
    uint64_t loc[PER], run = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      loc[j] = run;
      run = mc_scan_combine<OR_OP>(run, buf[threadIdx.x * PER + j]);
    }
    uint64_t tot;
    const uint64_t excl = mc_block_excl_scan<OR_OP>(run, red, &tot);
#pragma unroll
    for (int j = 0; j < PER; ++j)
      buf[threadIdx.x * PER + j] = mc_scan_combine<OR_OP>(carry, mc_scan_combine<OR_OP>(excl, loc[j]));
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const size_t i = r0 + (size_t)j * 1024 + threadIdx.x;
      if (i < ntiles) sums[i] = buf[j * 1024 + threadIdx.x];
    }
    carry = mc_scan_combine<OR_OP>(carry, tot);
    __syncthreads();
  }
}

template <bool OR_OP>
static inline void mc_launch_scan_sums(uint64_t *sums, size_t ntiles, hipStream_t st) {
  k_scan_sums<OR_OP><<<1, 1024, 0, st>>>(sums, ntiles);
}
