// mc_c4.hip -- fused FixedScaleOffset -> Delta -> Shuffle chunk pipeline
// (BASELINE configs[3]: FSO(offset, scale, f4 -> i2) -> Delta(i2) ->
// Shuffle(2)), the composition of fixedscaleoffset.py:83-113, delta.py:52-83
// and _shuffle.pyx:11-30 that a Zarr array with filters
// [FixedScaleOffset, Delta] and a shuffle applies per chunk.
//
// encode, one pass: each lane loads 4 consecutive float elements (and the
//   element before them), applies FSO encode exactly as numpy does it in the
//   float dtype (NEP 50: Python scalars are weak), takes wrap-around
//   differences in the integer dtype, and writes the 4 integers as plane
//   dwords of the shuffled chunk (4x4 byte transpose in registers).
//   HBM: read 4 (or 8) B + write 2 (or 4) B per element.
// decode, three passes over 4096-element tiles (mc_scan.h): per-tile totals
//   of the unshuffled deltas; exclusive scan of the totals (one workgroup);
//   rescan of each tile + FSO decode ((x / scale + offset) in float64, then
//   cast to the float dtype) + store.  HBM: read 2 B twice + write 4 B.
// Bit-exact with the reference sequence of codecs (tests/test_gpu_c4.py).
#include "mc_scan.h"
#include "mc_shuffle.h"

namespace {

struct C4Params {
  size_t n;      // elements
  McNum off;     // encode: offset in D;   decode: offset in f64
  McNum sc;      // encode: scale in D;    decode: scale in f64
};

template <int D, int A>
MC_DEV int64_t fso_enc(uint64_t xbits, const C4Params &p) {
  McNum v = mc_num_from_bits(xbits, D);
  v = mc_num_binop(v, p.off, MC_OP_SUB, D);
  v = mc_num_binop(v, p.sc, MC_OP_MUL, D);
  v = mc_num_rint(v, D);
  return mc_num_cast(v, D, A).i;
}

template <int D, int A>
MC_DEV uint64_t fso_dec(int64_t a, const C4Params &p) {
  McNum v = mc_num_cast(mc_num_i(a), A, MC_F8);
  v = mc_num_binop(v, p.sc, MC_OP_DIV, MC_F8);
  v = mc_num_binop(v, p.off, MC_OP_ADD, MC_F8);
  return mc_num_to_bits(mc_num_cast(v, MC_F8, D), D);
}

// pack 4 integers of width ES into the quad's ES dwords
template <int ES>
MC_DEV void pack_quad(const int64_t (&d)[4], uint32_t (&w)[ES]) {
  if constexpr (ES == 2) {
    w[0] = ((uint32_t)d[0] & 0xffffu) | ((uint32_t)d[1] << 16);
    w[1] = ((uint32_t)d[2] & 0xffffu) | ((uint32_t)d[3] << 16);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)d[k];
  }
}

template <int A, int ES>
MC_DEV void unpack_quad(const uint32_t (&w)[ES], int64_t (&d)[4]) {
  if constexpr (ES == 2) {
    d[0] = mc_wrap(w[0] & 0xffffu, A);
    d[1] = mc_wrap(w[0] >> 16, A);
    d[2] = mc_wrap(w[1] & 0xffffu, A);
    d[3] = mc_wrap(w[1] >> 16, A);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = mc_wrap(w[k], A);
  }
}

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_enc(const uint8_t *__restrict__ src,
                                                    uint8_t *__restrict__ dst, C4Params p) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  constexpr int DS = D == MC_F4 ? 4 : 8;
  const size_t tile_e0 = (size_t)blockIdx.x * MC_SCAN_TILE;
#pragma unroll
  for (int q = 0; q < MC_SCAN_STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    if (e >= p.n) continue;  // n % 4 == 0: quads are whole
    uint64_t x[4];
    mc_load4(src + e * DS, DS, x);
    int64_t a[4], d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = fso_enc<D, A>(x[k], p);
    if (e > 0) {
      const int64_t prev = fso_enc<D, A>(mc_load_elem(src, e - 1, DS), p);
      d[0] = mc_wrap(a[0] - prev, A);
    } else {
      d[0] = a[0];
    }
#pragma unroll
    for (int k = 1; k < 4; ++k) d[k] = mc_wrap(a[k] - a[k - 1], A);
    uint32_t w[ES], pl[ES];
    pack_quad<ES>(d, w);
    mc_quad_to_planes<ES>(w, pl);
#pragma unroll
    for (int b = 0; b < ES; ++b) mc_st4<true>(dst + (size_t)b * p.n + e, pl[b]);
  }
}

template <int A, int ES>
MC_DEV void load_deltas(const uint8_t *src, size_t n, size_t e, int64_t (&d)[4]) {
  uint32_t pl[ES], w[ES];
#pragma unroll
  for (int b = 0; b < ES; ++b) pl[b] = mc_ld4<true>(src + (size_t)b * n + e);
  mc_planes_to_quad<ES>(pl, w);
  unpack_quad<A, ES>(w, d);
}

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_reduce(const uint8_t *__restrict__ src,
                                                       uint64_t *__restrict__ sums, C4Params p) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const size_t tile_e0 = (size_t)blockIdx.x * MC_SCAN_TILE;
  uint64_t acc = 0;
#pragma unroll
  for (int q = 0; q < MC_SCAN_STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    if (e >= p.n) continue;
    int64_t d[4];
    load_deltas<A, ES>(src, p.n, e, d);
    acc += (uint64_t)(d[0] + d[1] + d[2] + d[3]);
  }
  uint64_t tot;
  mc_block_excl_scan<false>(acc, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_apply(const uint8_t *__restrict__ src,
                                                      uint8_t *__restrict__ dst,
                                                      const uint64_t *__restrict__ sums,
                                                      C4Params p) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  constexpr int DS = D == MC_F4 ? 4 : 8;
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const size_t tile_e0 = (size_t)blockIdx.x * MC_SCAN_TILE;
  uint64_t carry = sums[blockIdx.x];
#pragma unroll
  for (int q = 0; q < MC_SCAN_STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    const bool live = e < p.n;
    int64_t d[4] = {0, 0, 0, 0};
    if (live) load_deltas<A, ES>(src, p.n, e, d);
    uint64_t pr[4], run = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      run += (uint64_t)d[k];
      pr[k] = run;
    }
    uint64_t tot;
    const uint64_t excl = mc_block_excl_scan<false>(run, lds, &tot);  // all threads
    if (live) {
      const uint64_t pre = carry + excl;
      uint64_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = fso_dec<D, A>(mc_wrap((int64_t)(pre + pr[k]), A), p);
      if constexpr (DS == 4) {
        mc_st16<true>(dst + e * 4, mc_u32x4{(uint32_t)o[0], (uint32_t)o[1], (uint32_t)o[2], (uint32_t)o[3]});
      } else {
        mc_st16<true>(dst + e * 8, mc_u32x4{(uint32_t)o[0], (uint32_t)(o[0] >> 32), (uint32_t)o[1],
                                            (uint32_t)(o[1] >> 32)});
        mc_st16<true>(dst + e * 8 + 16, mc_u32x4{(uint32_t)o[2], (uint32_t)(o[2] >> 32),
                                                 (uint32_t)o[3], (uint32_t)(o[3] >> 32)});
      }
    }
    carry += tot;
  }
}

template <int D, int A>
static void c4_encode(const uint8_t *s, uint8_t *d, const C4Params &p, hipStream_t st) {
  const unsigned grid = (unsigned)((p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE);
  k_c4_enc<D, A><<<grid, MC_BLOCK, 0, st>>>(s, d, p);
}

template <int D, int A>
static void c4_decode(const uint8_t *s, uint8_t *d, uint64_t *sums, const C4Params &p,
                      hipStream_t st) {
  const size_t ntiles = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  k_c4_reduce<D, A><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, sums, p);
  mc_launch_scan_sums<false>(sums, ntiles, st);
  k_c4_apply<D, A><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, sums, p);
}

static bool c4_ok(const void *src, const void *dst, size_t n, int dtype, int astype) {
  if (!(dtype == MC_F4 || dtype == MC_F8)) return false;
  if (!(astype == MC_I2 || astype == MC_U2 || astype == MC_I4 || astype == MC_U4)) return false;
  if (n % 4 != 0) return false;
  return src && dst && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0;
}

#define MC_C4_DISPATCH(FN, ...)                                              \
  do {                                                                       \
    if (dtype == MC_F4) {                                                    \
      switch (astype) {                                                      \
        case MC_I2: FN<MC_F4, MC_I2>(__VA_ARGS__); break;                    \
        case MC_U2: FN<MC_F4, MC_U2>(__VA_ARGS__); break;                    \
        case MC_I4: FN<MC_F4, MC_I4>(__VA_ARGS__); break;                    \
        default: FN<MC_F4, MC_U4>(__VA_ARGS__); break;                       \
      }                                                                      \
    } else {                                                                 \
      switch (astype) {                                                      \
        case MC_I2: FN<MC_F8, MC_I2>(__VA_ARGS__); break;                    \
        case MC_U2: FN<MC_F8, MC_U2>(__VA_ARGS__); break;                    \
        case MC_I4: FN<MC_F8, MC_I4>(__VA_ARGS__); break;                    \
        default: FN<MC_F8, MC_U4>(__VA_ARGS__); break;                       \
      }                                                                      \
    }                                                                        \
  } while (0)

}  // namespace

extern "C" {

int mc_fso_delta_shuffle_encode(const void *src, void *dst, size_t n, int dtype, int astype,
                                double offset, double scale, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, dtype, astype)) return MC_EINVAL;
  C4Params p;
  p.n = n;
  p.off = mc_num_f(offset);
  p.sc = mc_num_f(scale);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  MC_C4_DISPATCH(c4_encode, s, d, p, st);
  return mc_last_launch();
}

size_t mc_fso_delta_shuffle_decode_workspace(size_t n) {
  return ((n + MC_SCAN_TILE - 1) / MC_SCAN_TILE) * sizeof(uint64_t);
}

int mc_fso_delta_shuffle_decode(const void *src, void *dst, size_t n, int astype, int dtype,
                                double scale, double offset, void *workspace,
                                size_t workspace_bytes, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, dtype, astype)) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_fso_delta_shuffle_decode_workspace(n)) return MC_ENOSPC;
  C4Params p;
  p.n = n;
  p.off = mc_num_f(offset);
  p.sc = mc_num_f(scale);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint64_t *sums = static_cast<uint64_t *>(workspace);
  hipStream_t st = (hipStream_t)stream;
  MC_C4_DISPATCH(c4_decode, s, d, sums, p, st);
  return mc_last_launch();
}

}  // extern "C"
