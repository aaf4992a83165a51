// mc_crc_bs.hip -- CRC32 / CRC32C tiles with the bit-sliced fold (see
// mc_crc_bs.h / gen_crc_bs.py for the derivation).  Separate translation unit
// from mc_checksum.hip so both template sets build in parallel.
#include "mc_checksum.h"

namespace mcck {
// ---------------------------------------------------------------------------
// CRC tiles with the bit-sliced fold (crc_fold_bs, K >= 4): no LDS tables;
// workgroups loop over tiles (grid: ck_grid_cap_bs) with the next tile's K
// vectors loaded into a second register set before the current tile is
// folded (the fold is ~3 VALU ops per byte, so with one tile per workgroup
// the loads and the XOR network of a workgroup serialise and ~half the wave
// time waited on memory).  Lane
// alignment x^(-128 l) uses the 32 products g * x^i kept in registers (one
// v_bitop3 + one v_bfe per bit); the four wave partials of a tile go through
// a parity-double-buffered LDS slot, one barrier per tile.
// ---------------------------------------------------------------------------
template <int KIND, int K, bool COPY, int ALS, int ALD, bool FUSED>
__global__ __launch_bounds__(MC_BLOCK, 2) void k_crc_tiles_bs(
    const uint8_t *__restrict__ src, size_t src_stride, uint8_t *__restrict__ dst,
    size_t dst_stride, size_t n, size_t tiles_per_chunk, size_t total_tiles,
    uint32_t *__restrict__ partials, const CrcFin fin, const CkFinish fx) {
  static_assert(KIND != K_ADLER && K >= 4, "bit-sliced folds exist for CRC tiles of 4, 8, 16 vectors");
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t gx[32];  // g * x^i, g = x^(-128 threadIdx.x)
  gx[0] = crc_consts<KIND>().g[threadIdx.x];
#pragma unroll
  for (int i = 1; i < 32; ++i) gx[i] = mulx_r<KIND>(gx[i - 1]);
  constexpr size_t TB = (size_t)K * STEP;
  auto load = [&](mc_u32x4 (&v)[K], size_t tile) {
    const size_t c = tile / tiles_per_chunk, t = tile - c * tiles_per_chunk;
    ck_load_tile<K, ALS>(v, src + c * src_stride, t * TB + 16 * (size_t)threadIdx.x, n, (t + 1) * TB <= n);
  };
  auto fold = [&](const mc_u32x4 (&v)[K], size_t tile, int par) {
    const size_t c = tile / tiles_per_chunk, t = tile - c * tiles_per_chunk;
    const size_t base = t * TB + 16 * (size_t)threadIdx.x;
    if constexpr (COPY) {
      uint8_t *d = dst + c * dst_stride;
      if ((t + 1) * TB <= n) {
#pragma unroll
        for (int k = 0; k < K; ++k) st_vec<ALD>(d + base + (size_t)k * STEP, v[k]);
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const size_t pos = base + (size_t)k * STEP;
          if (pos < n) st_masked<ALD>(d, pos, n, v[k]);
        }
      }
    }
    const uint32_t acc = crc_fold_bs<KIND, K>(v);
    uint32_t p = 0;  // acc * g: bit (31 - i) of acc selects g * x^i
#pragma unroll
    for (int i = 0; i < 32; ++i)
      p = __builtin_amdgcn_bitop3_b32(p, (uint32_t)__builtin_amdgcn_sbfe((int)acc, 31 - i, 1), gx[i], 0x78);
    p = wave_xor(p);
    if (lane == 0) red[par][wave] = p;
    __syncthreads();  // red[par] is rewritten two tiles later, after the next barrier
    if (threadIdx.x == 0) {
      uint32_t r = 0;
#pragma unroll
      for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= red[par][w];
      if constexpr (FUSED) __hip_atomic_store(&partials[tile], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else partials[tile] = r;
    }
  };
  mc_u32x4 a[K], b[K];
  size_t tile = blockIdx.x;
  if (tile < total_tiles) load(a, tile);
  while (tile < total_tiles) {
    const size_t t1 = tile + gridDim.x;
    if (t1 < total_tiles) load(b, t1);
    fold(a, tile, 0);
    if (t1 >= total_tiles) break;
    const size_t t2 = t1 + gridDim.x;
    if (t2 < total_tiles) load(a, t2);
    fold(b, t1, 1);
    tile = t2;
  }
  if constexpr (FUSED) ck_fused_tail<KIND, K>(fin, partials, tiles_per_chunk, n, src_stride, fx);
}

namespace {
template <int KIND, int K, bool COPY, int ALS, int ALD>
void launch_one(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t n, size_t tpc, size_t total,
                uint32_t *parts, const CrcFin &fin, const CkFinish *fx, unsigned grid, hipStream_t st) {
  if (fx)
    k_crc_tiles_bs<KIND, K, COPY, ALS, ALD, true><<<grid, MC_BLOCK, 0, st>>>(s, ss, d, ds, n, tpc, total, parts,
                                                                             fin, *fx);
  else
    k_crc_tiles_bs<KIND, K, COPY, ALS, ALD, false><<<grid, MC_BLOCK, 0, st>>>(s, ss, d, ds, n, tpc, total, parts,
                                                                              fin, CkFinish{});
}

template <int KIND, int K>
int launch_k(int als, int ald, const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t n, size_t tpc,
             size_t total, uint32_t *parts, const CrcFin &fin, const CkFinish *fx, unsigned grid, hipStream_t st) {
#define MC_BS_ARGS s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st
  if (!d) {
    if (als == 2) launch_one<KIND, K, false, 2, 2>(MC_BS_ARGS);
    else if (als == 1) launch_one<KIND, K, false, 1, 1>(MC_BS_ARGS);
    else launch_one<KIND, K, false, 0, 0>(MC_BS_ARGS);
  } else if (als == 2 && ald == 2) launch_one<KIND, K, true, 2, 2>(MC_BS_ARGS);
  else if (als == 1 && ald == 2) launch_one<KIND, K, true, 1, 2>(MC_BS_ARGS);
  else if (als == 2 && ald == 1) launch_one<KIND, K, true, 2, 1>(MC_BS_ARGS);
  else if (als >= 1 && ald >= 1) launch_one<KIND, K, true, 1, 1>(MC_BS_ARGS);
  else launch_one<KIND, K, true, 0, 0>(MC_BS_ARGS);
#undef MC_BS_ARGS
  return MC_OK;
}

template <int KIND>
int launch_kind(int K, int als, int ald, const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t n, size_t tpc,
                size_t total, uint32_t *parts, const CrcFin &fin, const CkFinish *fx, unsigned grid,
                hipStream_t st) {
  switch (K) {
    case 4: return launch_k<KIND, 4>(als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
    case 8: return launch_k<KIND, 8>(als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
    case 16: return launch_k<KIND, 16>(als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
    default: return MC_EINVAL;
  }
}
}  // namespace

int launch_crc_bs(int kind, int K, int als, int ald, const uint8_t *s, size_t ss, uint8_t *d, size_t ds,
                  size_t n, size_t tpc, size_t total, uint32_t *parts, const CrcFin &fin, const CkFinish *fx,
                  unsigned grid, hipStream_t st) {
  if (kind == MC_CK_CRC32)
    return launch_kind<K_CRC32>(K, als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
  if (kind == MC_CK_CRC32C)
    return launch_kind<K_CRC32C>(K, als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
  return MC_EINVAL;
}

}  // namespace mcck
