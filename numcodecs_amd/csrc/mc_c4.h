// mc_c4.h -- device helpers of the fused FSO -> Delta -> Shuffle chunk
// pipeline (mc_c4.hip), shared with the lab's alternative decode schedules
// (tools/lab/lab_c4.hip).  fixedscaleoffset.py:83-113, delta.py:52-83,
// _shuffle.pyx:11-30.
#pragma once

#include "mc_scan.h"
#include "mc_shuffle.h"

namespace {

struct C4Params {
  size_t n;      // elements
  McNum off;     // encode: offset in D;   decode: offset in f64
  McNum sc;      // encode: scale in D;    decode: scale in f64
  double rcp;    // decode: RN(1 / scale), computed on the host
  bool fastdiv;  // decode: divide by scale as mul + 2 FMA (mc_div_by_const)
};

// decode parameters: offset/scale in float64 (numpy promotes the int16
// array / Python float to float64, fixedscaleoffset.py:107-110) and the
// host-rounded reciprocal for the exact constant division (mc_div_by_const)
static inline C4Params c4_decode_params(size_t n, double scale, double offset) {
  C4Params p;
  p.n = n;
  p.off = mc_num_f(offset);
  p.sc = mc_num_f(scale);
  p.rcp = 1.0 / scale;
  p.fastdiv = mc_fastdiv_ok(scale);
  return p;
}

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
  if (p.fastdiv) v = mc_num_f(mc_div_by_const(v.f, p.sc.f, p.rcp));
  else v = mc_num_binop(v, p.sc, MC_OP_DIV, MC_F8);
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

// A thread owns 16 consecutive elements of a 4096-element tile: one 16-B
// (lane-contiguous) load per plane, 4 quads unshuffled in registers.
constexpr int C4_PER = 16;

// the 16 deltas of one unit from its ES plane vectors (dword c of every
// plane = elements 4c..4c+3), as astype values widened to 32 bits
template <int A, int ES>
MC_DEV void c4_planes_to_deltas(const mc_u32x4 (&pl)[ES], uint32_t (&v)[C4_PER]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    uint32_t pq[ES], w[ES];
#pragma unroll
    for (int b = 0; b < ES; ++b) pq[b] = pl[b][c];
    mc_planes_to_quad<ES>(pq, w);
    int64_t d[4];
    unpack_quad<A, ES>(w, d);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[4 * c + k] = (uint32_t)d[k];
  }
}

// NT: nontemporal loads (the 3-pass scan); the two-launch decode loads with
// the default policy so that the apply pass's re-read hits the Infinity Cache
template <int A, int ES, bool NT = true>
MC_DEV void load16_deltas(const uint8_t *src, size_t n, size_t e0, uint32_t (&v)[C4_PER]) {
  mc_u32x4 pl[ES];
#pragma unroll
  for (int b = 0; b < ES; ++b) pl[b] = mc_ld16<NT>(src + (size_t)b * n + e0);
  c4_planes_to_deltas<A, ES>(pl, v);
}

// scan of 16 consecutive deltas + FSO decode, staged through LDS for
// lane-contiguous 16-B stores; `pre` = exclusive prefix of the thread.
// The staging image is addressed in 16-B units with unit u stored at
// u ^ ((u >> 3) & 7): a thread's own DS units (written with ds_write_b128,
// 8-lane groups) and the lane-contiguous read-back (ds_read_b128, 16-lane
// groups) are then both conflict-free.  Unswizzled, the 16 ds_write_b32 per
// thread at a 64-B lane stride were 16-way bank conflicts.
MC_DEV int c4_swz(int u) { return u ^ ((u >> 3) & 7); }

template <int D, int A>
MC_DEV void c4_finish(uint8_t *dst, size_t tile, const uint32_t (&incl)[C4_PER], uint32_t pre,
                      uint8_t *outb, const C4Params &p) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  constexpr int UPT = C4_PER * DS / 16;  // 16-B units per thread
  mc_u32x4 *img = reinterpret_cast<mc_u32x4 *>(outb);
  uint32_t o[C4_PER * DS / 4];
#pragma unroll
  for (int k = 0; k < C4_PER; ++k) {
    const uint64_t x = fso_dec<D, A>(mc_wrap((int64_t)(uint32_t)(pre + incl[k]), A), p);
    if constexpr (DS == 4) {
      o[k] = (uint32_t)x;
    } else {
      o[2 * k] = (uint32_t)x;
      o[2 * k + 1] = (uint32_t)(x >> 32);
    }
  }
#pragma unroll
  for (int j = 0; j < UPT; ++j)
    img[c4_swz((int)threadIdx.x * UPT + j)] = mc_u32x4{o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]};
  __syncthreads();
  const size_t tile_b0 = tile * (size_t)MC_SCAN_TILE * DS;
  const size_t nbytes = p.n * DS;
#pragma unroll
  for (int r = 0; r < MC_SCAN_TILE * DS / 16 / MC_BLOCK; ++r) {
    const int u = r * MC_BLOCK + (int)threadIdx.x;
    const size_t off = (size_t)u * 16;
    if (tile_b0 + off < nbytes) mc_st16<true>(dst + tile_b0 + off, img[c4_swz(u)]);
  }
}

template <int D, int A>
MC_DEV void c4_local_scan(const uint8_t *src, size_t tile, const C4Params &p, uint32_t (&v)[C4_PER],
                          uint32_t &run) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  if (e0 < p.n) {
    load16_deltas<A, ES>(src, p.n, e0, v);
  } else {
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) v[k] = 0;
  }
  run = 0;
#pragma unroll
  for (int k = 0; k < C4_PER; ++k) {
    run += v[k];
    v[k] = run;
  }
}

template <int A>
constexpr int c4_es() { return A == MC_I2 || A == MC_U2 ? 2 : 4; }

static inline bool c4_ok(const void *src, const void *dst, size_t n, int dtype, int astype) {
  if (!(dtype == MC_F4 || dtype == MC_F8)) return false;
  if (!(astype == MC_I2 || astype == MC_U2 || astype == MC_I4 || astype == MC_U4)) return false;
  if (n % 16 != 0) return false;  // 16-B plane accesses (decode)
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
