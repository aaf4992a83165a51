// mc_crc_bs.hip -- CRC32 / CRC32C tiles with the bit-sliced fold (see
// mc_crc_bs.h / gen_crc_bs.py for the derivation).  Separate translation unit
// from mc_checksum.hip so both template sets build in parallel.
#include "mc_checksum.h"

namespace mcck {
// ---------------------------------------------------------------------------
// CRC tiles with the bit-sliced fold (mc_crc_bs.h, K >= 4): no slicing
// tables, a persistent grid, and the next tile's vectors loaded while the
// current tile is folded -- in two halves: the first half at the start of
// the fold, the second once the network has consumed the current tile's
// first half, so the two tiles share 1.5 register sets (the fold is ~3 VALU
// ops per byte: with one tile per workgroup the loads and the XOR network
// of a workgroup serialise; with a full second register set the kernel needs
// 228 VGPRs, two waves per SIMD).  Lane alignment: the lane's raw CRC times
// x^(-128 l) through per-lane nibble tables in LDS (8 conflict-free
// ds_read_b32: entry (j, nib) of lane l at dword (16 j + nib) * 64 + l), the
// wave's sum times x^(-128 * 64 w) through a broadcast table; the four wave
// partials of a tile pass through a parity-double-buffered LDS slot, one
// barrier per tile.
// ---------------------------------------------------------------------------
template <int KIND, int K, int PART>
MC_DEV void crc_bs_part(uint32_t (&w)[32], const mc_u32x4 *v) {
  if constexpr (KIND == K_CRC32C) {
    if constexpr (K == 4) PART ? crc_bs_crc32c_k4_part1(w, v) : crc_bs_crc32c_k4_part0(w, v);
    else if constexpr (K == 8) PART ? crc_bs_crc32c_k8_part1(w, v) : crc_bs_crc32c_k8_part0(w, v);
    else PART ? crc_bs_crc32c_k16_part1(w, v) : crc_bs_crc32c_k16_part0(w, v);
  } else {
    if constexpr (K == 4) PART ? crc_bs_crc32_k4_part1(w, v) : crc_bs_crc32_k4_part0(w, v);
    else if constexpr (K == 8) PART ? crc_bs_crc32_k8_part1(w, v) : crc_bs_crc32_k8_part0(w, v);
    else PART ? crc_bs_crc32_k16_part1(w, v) : crc_bs_crc32_k16_part0(w, v);
  }
}
template <int KIND>
MC_DEV uint32_t crc_bs_horner(const uint32_t (&w)[32]) {
  if constexpr (KIND == K_CRC32C) return crc_bs_horner_crc32c(w);
  else return crc_bs_horner_crc32(w);
}

// vectors [LO, HI) of a tile (bytes past n read as zero)
template <int K, int LO, int HI, int ALS>
MC_DEV void ck_load_range(mc_u32x4 (&v)[K], const uint8_t *s, size_t base, size_t n, bool full) {
  if (full) {
#pragma unroll
    for (int k = LO; k < HI; ++k) v[k] = ld_vec<ALS>(s + base + (size_t)k * STEP);
  } else {
#pragma unroll
    for (int k = LO; k < HI; ++k) {
      const size_t pos = base + (size_t)k * STEP;
      v[k] = pos < n ? ld_masked<ALS>(s, pos, n) : mc_u32x4{0, 0, 0, 0};
    }
  }
}

template <int KIND, int K, bool COPY, int ALS, int ALD, bool FUSED>
__global__ __launch_bounds__(MC_BLOCK, 2) void k_crc_tiles_bs(
    const uint8_t *__restrict__ src, size_t src_stride, uint8_t *__restrict__ dst,
    size_t dst_stride, size_t n, size_t tiles_per_chunk, size_t total_tiles,
    uint32_t *__restrict__ partials, const CrcFin fin, const CkFinish fx) {
  static_assert(KIND != K_ADLER && K >= 4, "bit-sliced folds exist for CRC tiles of 4, 8, 16 vectors");
  constexpr int NW = MC_BLOCK / 64;
  __shared__ uint32_t red[2][NW];
  __shared__ uint32_t lt[8 * 16 * 64];  // lane l: g_l * (nibble j of acc), g_l = x^(-128 l)
  __shared__ uint32_t wt[NW * 8 * 16];  // wave w: G_w * (nibble j), G_w = x^(-128 * 64 w)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {
    // nibble j of a 32-bit value = bits 28-4j .. 31-4j = coefficients x^(4j+3) .. x^(4j)
    uint32_t b = crc_consts<KIND>().g[lane];
    for (int i = 0; i < 8 * wave; ++i) b = mulx_r<KIND>(b);  // g * x^(4j), j = 2 * wave
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = 2 * wave + jj;
      uint32_t e[4];  // e[bit] = g * x^(4j + 3 - bit)
      e[3] = b;
      e[2] = mulx_r<KIND>(e[3]);
      e[1] = mulx_r<KIND>(e[2]);
      e[0] = mulx_r<KIND>(e[1]);
#pragma unroll
      for (int nib = 0; nib < 16; ++nib)
        lt[(j * 16 + nib) * 64 + lane] = ((nib & 1) ? e[0] : 0u) ^ ((nib & 2) ? e[1] : 0u) ^
                                         ((nib & 4) ? e[2] : 0u) ^ ((nib & 8) ? e[3] : 0u);
      b = mulx_r<KIND>(e[0]);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int ent = threadIdx.x + r * MC_BLOCK;  // (w * 8 + j) * 16 + nib
      const uint32_t poly_bits = (uint32_t)(ent & 15) << (28 - 4 * ((ent >> 4) & 7));
      wt[ent] = gf_mul(poly_bits, crc_consts<KIND>().g[64 * (ent >> 7)], crc_poly<KIND>());
    }
    __syncthreads();
  }
  constexpr size_t TB = (size_t)K * STEP;
  constexpr int H = K / 2;
  auto fold = [&](const mc_u32x4 (&v)[K], mc_u32x4 (&nv)[K], size_t tile, size_t next, int par) {
    const size_t c = tile / tiles_per_chunk, t = tile - c * tiles_per_chunk;
    const size_t base = t * TB + 16 * (size_t)threadIdx.x;
    const size_t nc = next / tiles_per_chunk, nt = next - nc * tiles_per_chunk;
    const uint8_t *ns = src + nc * src_stride;
    const size_t nbase = nt * TB + 16 * (size_t)threadIdx.x;
    const bool nfull = (nt + 1) * TB <= n;
    const bool more = next < total_tiles;
    if (more) ck_load_range<K, 0, H, ALS>(nv, ns, nbase, n, nfull);
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
    uint32_t w[32];
    crc_bs_part<KIND, K, 0>(w, v);
    if (more) ck_load_range<K, H, K, ALS>(nv, ns, nbase, n, nfull);  // into the registers just freed
    crc_bs_part<KIND, K, 1>(w, v);
    const uint32_t acc = crc_bs_horner<KIND>(w);
    uint32_t p = 0;  // acc * g_lane
#pragma unroll
    for (int j = 0; j < 8; ++j) p ^= lt[(j * 16 + ((acc >> (28 - 4 * j)) & 15u)) * 64 + lane];
    p = wave_xor(p);
    uint32_t q = 0;  // * G_wave (wave-uniform: broadcast reads)
#pragma unroll
    for (int j = 0; j < 8; ++j) q ^= wt[(wave * 8 + j) * 16 + ((p >> (28 - 4 * j)) & 15u)];
    if (lane == 0) red[par][wave] = q;
    __syncthreads();  // red[par] is rewritten two tiles later, after the next barrier
    if (threadIdx.x == 0) {
      uint32_t r = 0;
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) r ^= red[par][w2];
      if constexpr (FUSED) __hip_atomic_store(&partials[tile], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else partials[tile] = r;
    }
  };
  mc_u32x4 a[K], b[K];
  size_t tile = blockIdx.x;
  if (tile < total_tiles) {
    const size_t c = tile / tiles_per_chunk, t = tile - c * tiles_per_chunk;
    ck_load_range<K, 0, K, ALS>(a, src + c * src_stride, t * TB + 16 * (size_t)threadIdx.x, n, (t + 1) * TB <= n);
  }
  while (tile < total_tiles) {
    const size_t t1 = tile + gridDim.x;
    fold(a, b, tile, t1, 0);
    if (t1 >= total_tiles) break;
    const size_t t2 = t1 + gridDim.x;
    fold(b, a, t1, t2, 1);
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
