// mc_crc_bs.hip -- CRC32 / CRC32C tiles with the bit-sliced fold (see
// mc_crc_bs.h / gen_crc_bs.py for the derivation).  Separate translation unit
// from mc_checksum.hip so both template sets build in parallel.
#include "mc_checksum.h"

namespace mcck {
// X^e, X = x^(8 * K * STEP), for e < CK_RIDE_MAX_GRID: the one-launch
// finish's shift of workgroup b's last tile to the chunk end, e = (tiles - 1
// - b) mod G (built by the compiler, one table per CRC and tile size)
struct CkRidePow {
  uint32_t p[CK_RIDE_MAX_GRID];
};
constexpr CkRidePow make_ride_pow(uint32_t poly, int K) {
  CkRidePow t{};
  uint32_t x2n[64] = {};
  x2n[0] = GF_X;
  for (int k = 1; k < 64; ++k) x2n[k] = gf_mul(x2n[k - 1], x2n[k - 1], poly);
  const uint32_t X = xpow_tab(x2n, 8ull * K * STEP, poly);
  t.p[0] = GF_ONE;
  for (unsigned e = 1; e < CK_RIDE_MAX_GRID; ++e) t.p[e] = gf_mul(t.p[e - 1], X, poly);
  return t;
}
static __constant__ const CkRidePow kRide32[3] = {make_ride_pow(POLY_CRC32, 4), make_ride_pow(POLY_CRC32, 8),
                                                  make_ride_pow(POLY_CRC32, 16)};
static __constant__ const CkRidePow kRide32c[3] = {make_ride_pow(POLY_CRC32C, 4), make_ride_pow(POLY_CRC32C, 8),
                                                   make_ride_pow(POLY_CRC32C, 16)};
template <int KIND, int K>
MC_DEV const CkRidePow &ride_pow() {
  constexpr int i = K == 4 ? 0 : K == 8 ? 1 : 2;
  if constexpr (KIND == K_CRC32C) return kRide32c[i];
  else return kRide32[i];
}

// ---------------------------------------------------------------------------
// CRC tiles with the bit-sliced fold (crc_fold_bs, K >= 4): no LDS tables;
// workgroups loop over tiles (grid: ck_bs_grid) with the next tile's K
// vectors loaded into a second register set before the current tile is
// folded (the fold is ~3 VALU ops per byte, so with one tile per workgroup
// the loads and the XOR network of a workgroup serialise and ~half the wave
// time waited on memory).  Lane
// alignment x^(-128 l) uses the 32 products g * x^i kept in registers (one
// v_bitop3 + one v_bfe per bit); the four wave partials of a tile go through
// a parity-double-buffered LDS slot, one barrier per tile.
// FUSED (one chunk, grid <= CK_RIDE_MAX_GRID): no partial stores.  The lane
// alignment constant also carries the workgroup's shift to the chunk end
// (g * X^e, e = (tiles - 1 - b) mod G), so its tile sums come out shifted;
// wave 0 sums them by Horner with X^G on the scalar unit (the basis in the
// kernel arguments) and arrives through ck_ride_arrive.
// ---------------------------------------------------------------------------
template <int KIND, int K, bool COPY, int ALS, int ALD, bool FUSED>
__global__ __launch_bounds__(MC_BLOCK, 2) void k_crc_tiles_bs(
    const uint8_t *__restrict__ src, size_t src_stride, uint8_t *__restrict__ dst,
    size_t dst_stride, size_t n, size_t tiles_per_chunk, size_t total_tiles,
    uint32_t *__restrict__ partials, const CrcFin fin, const CkFinish fx) {
  static_assert(KIND != K_ADLER && K >= 4, "bit-sliced folds exist for CRC tiles of 4, 8, 16 vectors");
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t gx[32];  // g * x^i, g = x^(-128 threadIdx.x) (FUSED: times the workgroup's shift)
  constexpr size_t TB = (size_t)K * STEP;
  constexpr uint32_t poly = crc_poly<KIND>();
  uint32_t hz = 0;  // FUSED, wave 0: sum over this workgroup's tiles so far (wave-uniform)
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
    if constexpr (FUSED) {
      if (__builtin_amdgcn_readfirstlane(wave) == 0) {  // (wave-uniform: the sum stays scalar)
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= red[par][w];
        uint32_t m = 0;  // hz * X^G
#pragma unroll
        for (int i = 0; i < 32; ++i) m ^= ((hz >> i) & 1u) ? fin.xgb[i] : 0u;
        hz = m ^ __builtin_amdgcn_readfirstlane(r);
      }
    } else if (threadIdx.x == 0) {
      uint32_t r = 0;
#pragma unroll
      for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= red[par][w];
      partials[tile] = r;
    }
  };
  mc_u32x4 a[K], b[K];
  size_t tile = blockIdx.x;
  if (tile < total_tiles) load(a, tile);
  // while the first tile loads: the lane constants, and for the finish the
  // stored word, each byte in a register of its own and nothing computed
  // from them until the finish -- a use here waits for every load issued
  // before (the tile's too: vmcnt counts in order), and the next tile's loads
  // would issue only after the first tile arrived (tools/probe_ck_tail.py:
  // a tail folded this way instead of a ragged last tile took 47 -> 58 us)
  uint32_t g = crc_consts<KIND>().g[threadIdx.x];
  uint32_t hb[4] = {0, 0, 0, 0};
  if constexpr (FUSED) {
    g = gf_mul(ride_pow<KIND, K>().p[(total_tiles - 1 - blockIdx.x) % gridDim.x], g, poly);
    if (threadIdx.x == 0 && fx.stored) {
#pragma unroll
      for (int j = 0; j < 4; ++j) hb[j] = fx.stored[j];
    }
  }
  gx[0] = g;
#pragma unroll
  for (int i = 1; i < 32; ++i) gx[i] = mulx_r<KIND>(gx[i - 1]);
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
  if constexpr (FUSED)
    if (threadIdx.x == 0 && ck_ride_arrive(fx.ticket, hz)) ck_ride_finish<KIND>(fin, fx, hz, hb);
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
  // the one-launch encode's payload copy to an aligned destination: the
  // dword-aligned (plain) 16-B store variant when ck_fused_plain is set
  if (fx && d && ald == 2 && mc_sched.ck_fused_plain) ald = 1;
  if (kind == MC_CK_CRC32)
    return launch_kind<K_CRC32>(K, als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
  if (kind == MC_CK_CRC32C)
    return launch_kind<K_CRC32C>(K, als, ald, s, ss, d, ds, n, tpc, total, parts, fin, fx, grid, st);
  return MC_EINVAL;
}

}  // namespace mcck
