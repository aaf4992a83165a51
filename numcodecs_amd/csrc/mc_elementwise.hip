// mc_elementwise.hip -- fused per-element codecs for gfx950.
//
//   mc_bitround   bitround.py:45-69   (integer ops on the same-width view)
//   mc_fso_encode fixedscaleoffset.py:83-97   astype(rint((x - offset) * scale))
//   mc_fso_decode fixedscaleoffset.py:99-113  dtype(x / scale + offset)
//   mc_quantize   quantize.py:60-76   astype(rint(scale * x) / scale)
//   mc_cast       ndarray.astype (quantize.py:80, compat.py:177-206)
//   mc_delta_encode delta.py:52-67     x[0], np.diff(x)
//
// Each numpy expression of the reference is one pass over HBM here (the
// reference makes 2-5 full-array temporaries).  Lanes move 4 consecutive
// elements per step with one vector access (lane-contiguous across the wave);
// a thread does STEPS steps, so a workgroup covers 4*STEPS*256 elements and
// the grid covers the whole array (no grid-stride loop: see mc_shuffle.hip on
// why looping workgroups lose to one-tile-per-workgroup).  Scalars arrive
// already converted to their compute dtype by the host (NEP 50 rules).
#include "mc_num.h"

namespace {

constexpr int STEPS = 4;
constexpr int ELEMS_PER_BLOCK = 4 * STEPS * MC_BLOCK;  // 4096

enum MapKind { K_CAST = 0, K_FSO_ENC = 1, K_FSO_DEC = 2, K_QUANTIZE = 3 };

struct MapParams {
  int d, t1, t2, a;  // input dtype, compute dtypes, output dtype
  McNum s0, s1;      // scalars in their compute dtypes
  double rcp = 0.0;      // FSO decode: RN(1 / scale) (host)
  bool fastdiv = false;  // FSO decode: integer input, f64 division by the constant scale
};

template <int KIND>
MC_DEV McNum map_op(McNum x, int d, int t1, int t2, int a, const McNum &s0, const McNum &s1,
                    double rcp = 0.0, bool fastdiv = false) {
  if constexpr (KIND == K_CAST) {
    return mc_num_cast(x, d, a);
  } else if constexpr (KIND == K_FSO_ENC) {  // s0 = offset (t1), s1 = scale (t2)
    McNum v = mc_num_cast(x, d, t1);
    v = mc_num_binop(v, s0, MC_OP_SUB, t1);
    v = mc_num_cast(v, t1, t2);
    v = mc_num_binop(v, s1, MC_OP_MUL, t2);
    v = mc_num_rint(v, t2);
    return mc_num_cast(v, t2, a);
  } else if constexpr (KIND == K_FSO_DEC) {  // s0 = scale (t1), s1 = offset (t2)
    McNum v = mc_num_cast(x, d, t1);
    if (fastdiv) v = mc_num_f(mc_div_by_const(v.f, s0.f, rcp));  // t1 == f64, integer x
    else v = mc_num_binop(v, s0, MC_OP_DIV, t1);
    v = mc_num_cast(v, t1, t2);
    v = mc_num_binop(v, s1, MC_OP_ADD, t2);
    return mc_num_cast(v, t2, a);
  } else {  // K_QUANTIZE: s0 = scale (d)
    McNum v = mc_num_cast(x, d, d);
    v = mc_num_binop(s0, v, MC_OP_MUL, d);
    v = mc_num_rint(v, d);
    v = mc_num_binop(v, s0, MC_OP_DIV, d);
    return mc_num_cast(v, d, a);
  }
}

// D_/T1_/T2_/A_ >= 0: compile-time dtypes (specialised hot paths); -1: runtime.
// EPL = elements per lane per step: 4, or 2 when one side is 8-B elements,
// so that the wide side moves one lane-contiguous 16-B vector per lane.
template <int KIND, int D_, int T1_, int T2_, int A_, bool VEC, int EPL = 4>
__global__ __launch_bounds__(MC_BLOCK) void k_map(const uint8_t *__restrict__ src,
                                                  uint8_t *__restrict__ dst, size_t n,
                                                  MapParams prm) {
  const int d = D_ >= 0 ? D_ : prm.d;
  const int t1 = T1_ >= 0 ? T1_ : prm.t1;
  const int t2 = T2_ >= 0 ? T2_ : prm.t2;
  const int a = A_ >= 0 ? A_ : prm.a;
  const int ss = mc_itemsize(d), ds = mc_itemsize(a);
  const size_t base = (size_t)blockIdx.x * ELEMS_PER_BLOCK;
  auto op = [&](uint64_t e) {
    return mc_num_to_bits(map_op<KIND>(mc_num_from_bits(e, d), d, t1, t2, a, prm.s0, prm.s1, prm.rcp, prm.fastdiv), a);
  };
  if (VEC && base + ELEMS_PER_BLOCK <= n) {
    // whole block in range: every load of the block issued before any store;
    // nontemporal accesses (streamed once)
    constexpr int NS = EPL == 2 ? 2 * STEPS : STEPS;
    uint64_t e[NS][EPL];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const size_t i0 = base + (size_t)s * EPL * MC_BLOCK + EPL * (size_t)threadIdx.x;
      if constexpr (EPL == 2) mc_load2<true>(src + i0 * ss, ss, e[s]);
      else mc_load4<true>(src + i0 * ss, ss, e[s]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const size_t i0 = base + (size_t)s * EPL * MC_BLOCK + EPL * (size_t)threadIdx.x;
      uint64_t o[EPL];
#pragma unroll
      for (int k = 0; k < EPL; ++k) o[k] = op(e[s][k]);
      if constexpr (EPL == 2) mc_store2<true>(dst + i0 * ds, ds, o);
      else mc_store4<true>(dst + i0 * ds, ds, o);
    }
    return;
  }
  if constexpr (VEC && EPL == 2) {
#pragma unroll
    for (int s = 0; s < 2 * STEPS; ++s) {
      const size_t i0 = base + (size_t)s * 2 * MC_BLOCK + 2 * (size_t)threadIdx.x;
      if (i0 + 2 <= n) {
        uint64_t e[2], o[2];
        mc_load2(src + i0 * ss, ss, e);
#pragma unroll
        for (int k = 0; k < 2; ++k)
          o[k] = mc_num_to_bits(map_op<KIND>(mc_num_from_bits(e[k], d), d, t1, t2, a, prm.s0, prm.s1, prm.rcp, prm.fastdiv), a);
        mc_store2(dst + i0 * ds, ds, o);
      } else if (i0 < n) {
        mc_store_elem(dst, i0, ds,
                      mc_num_to_bits(map_op<KIND>(mc_num_from_bits(mc_load_elem(src, i0, ss), d),
                                                  d, t1, t2, a, prm.s0, prm.s1, prm.rcp, prm.fastdiv), a));
      }
    }
  } else if constexpr (VEC) {
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const size_t i0 = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
      if (i0 + 4 <= n) {
        uint64_t e[4], o[4];
        mc_load4(src + i0 * ss, ss, e);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          o[k] = mc_num_to_bits(map_op<KIND>(mc_num_from_bits(e[k], d), d, t1, t2, a, prm.s0, prm.s1, prm.rcp, prm.fastdiv), a);
        mc_store4(dst + i0 * ds, ds, o);
      } else {
        for (size_t i = i0; i < n; ++i)
          mc_store_elem(dst, i, ds,
                        mc_num_to_bits(map_op<KIND>(mc_num_from_bits(mc_load_elem(src, i, ss), d),
                                                    d, t1, t2, a, prm.s0, prm.s1, prm.rcp, prm.fastdiv), a));
      }
    }
  } else {
    for (size_t i = base + threadIdx.x; i < n && i < base + ELEMS_PER_BLOCK; i += MC_BLOCK)
      mc_store_elem_u(dst, i, ds,
                      mc_num_to_bits(map_op<KIND>(mc_num_from_bits(mc_load_elem_u(src, i, ss), d),
                                                  d, t1, t2, a, prm.s0, prm.s1, prm.rcp, prm.fastdiv), a));
  }
}

// ---------------------------------------------------------------------------
// BitRound (bitround.py:62-68) on 16-B vectors
// ---------------------------------------------------------------------------
template <int ES>
__global__ __launch_bounds__(MC_BLOCK) void k_bitround(const uint8_t *__restrict__ src,
                                                       uint8_t *__restrict__ dst, size_t nbytes,
                                                       McBitRound br, bool vec) {
  const size_t base = (size_t)blockIdx.x * (16 * STEPS * MC_BLOCK);
  auto round4 = [&](mc_u32x4 v) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if constexpr (ES == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = mc_bitround16x2(w[k], br);
    } else if constexpr (ES == 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = mc_bitround32(w[k], br);
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint64_t r = mc_bitround64(((uint64_t)w[2 * k + 1] << 32) | w[2 * k], br);
        w[2 * k] = (uint32_t)r;
        w[2 * k + 1] = (uint32_t)(r >> 32);
      }
    }
    return mc_u32x4{w[0], w[1], w[2], w[3]};
  };
  if (vec && base + 16 * STEPS * MC_BLOCK <= nbytes) {
    // whole block in range: every load issued before any store
    mc_u32x4 v[STEPS];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) v[s] = mc_ld16<true>(src + base + ((size_t)s * MC_BLOCK + threadIdx.x) * 16);
#pragma unroll
    for (int s = 0; s < STEPS; ++s)
      mc_st16<true>(dst + base + ((size_t)s * MC_BLOCK + threadIdx.x) * 16, round4(v[s]));
    return;
  }
  if (vec) {
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const size_t o = base + ((size_t)s * MC_BLOCK + threadIdx.x) * 16;
      if (o + 16 <= nbytes) {
        mc_u32x4 v = mc_ld16<true>(src + o);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        if constexpr (ES == 2) {
#pragma unroll
          for (int k = 0; k < 4; ++k) w[k] = mc_bitround16x2(w[k], br);
        } else if constexpr (ES == 4) {
#pragma unroll
          for (int k = 0; k < 4; ++k) w[k] = mc_bitround32(w[k], br);
        } else {
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const uint64_t r = mc_bitround64(((uint64_t)w[2 * k + 1] << 32) | w[2 * k], br);
            w[2 * k] = (uint32_t)r;
            w[2 * k + 1] = (uint32_t)(r >> 32);
          }
        }
        mc_st16<true>(dst + o, mc_u32x4{w[0], w[1], w[2], w[3]});
      } else if (o < nbytes) {  // tail: whole elements, byte-wise
        for (size_t e = o; e + ES <= nbytes; e += ES) {
          uint64_t v = mc_load_elem_u(src + e, 0, ES);
          v = ES == 2 ? (mc_bitround16x2((uint32_t)v, br) & 0xffffu)
              : ES == 4 ? mc_bitround32((uint32_t)v, br) : mc_bitround64(v, br);
          mc_store_elem_u(dst + e, 0, ES, v);
        }
      }
    }
  } else {
    const size_t per = 16 * STEPS * MC_BLOCK;
    for (size_t e = base + (size_t)threadIdx.x * ES; e + ES <= nbytes && e < base + per;
         e += (size_t)MC_BLOCK * ES) {
      uint64_t v = mc_load_elem_u(src + e, 0, ES);
      v = ES == 2 ? (mc_bitround16x2((uint32_t)v, br) & 0xffffu)
          : ES == 4 ? mc_bitround32((uint32_t)v, br) : mc_bitround64(v, br);
      mc_store_elem_u(dst + e, 0, ES, v);
    }
  }
}

// ---------------------------------------------------------------------------
// Delta encode (delta.py:52-67): y[0] = astype(x[0]); y[i] = astype(x[i] - x[i-1])
// with the difference computed in dtype (bool: not_equal, as np.diff does).
// ---------------------------------------------------------------------------
template <int D_, int A_, bool VEC>
__global__ __launch_bounds__(MC_BLOCK) void k_delta_enc(const uint8_t *__restrict__ src,
                                                        uint8_t *__restrict__ dst, size_t n,
                                                        int d_rt, int a_rt, size_t src_stride,
                                                        size_t dst_stride) {
  src += (size_t)blockIdx.y * src_stride;  // chunk blockIdx.y of a batch
  dst += (size_t)blockIdx.y * dst_stride;
  const int d = D_ >= 0 ? D_ : d_rt;
  const int a = A_ >= 0 ? A_ : a_rt;
  const int ss = mc_itemsize(d), ds = mc_itemsize(a);
  const size_t base = (size_t)blockIdx.x * ELEMS_PER_BLOCK;
  auto diff = [&](McNum cur, McNum prev) {
    return mc_num_cast(mc_num_binop(cur, prev, MC_OP_SUB, d), d, a);
  };
  if constexpr (VEC) {
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const size_t i0 = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
      if (i0 + 4 <= n) {
        uint64_t e[4], o[4];
        mc_load4(src + i0 * ss, ss, e);
        McNum x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = mc_num_from_bits(e[k], d);
        const McNum prev = i0 ? mc_num_from_bits(mc_load_elem(src, i0 - 1, ss), d) : x[0];
        o[0] = mc_num_to_bits(i0 ? diff(x[0], prev) : mc_num_cast(x[0], d, a), a);
#pragma unroll
        for (int k = 1; k < 4; ++k) o[k] = mc_num_to_bits(diff(x[k], x[k - 1]), a);
        mc_store4(dst + i0 * ds, ds, o);
      } else {
        for (size_t i = i0; i < n; ++i) {
          const McNum x = mc_num_from_bits(mc_load_elem(src, i, ss), d);
          const McNum r = i ? diff(x, mc_num_from_bits(mc_load_elem(src, i - 1, ss), d))
                            : mc_num_cast(x, d, a);
          mc_store_elem(dst, i, ds, mc_num_to_bits(r, a));
        }
      }
    }
  } else {
    for (size_t i = base + threadIdx.x; i < n && i < base + ELEMS_PER_BLOCK; i += MC_BLOCK) {
      const McNum x = mc_num_from_bits(mc_load_elem_u(src, i, ss), d);
      const McNum r = i ? diff(x, mc_num_from_bits(mc_load_elem_u(src, i - 1, ss), d))
                        : mc_num_cast(x, d, a);
      mc_store_elem_u(dst, i, ds, mc_num_to_bits(r, a));
    }
  }
}

// Same-width integer Delta encode on 16-B vectors (astype == dtype, 16-B
// aligned rows).  Wrapping differences are bit operations on the packed
// vector: the "previous element" vector is the vector shifted up by one
// element (v_alignbit with the dword before it, which comes from the lane
// below by a shuffle, or from memory for lane 0 of a wave), and the packed
// subtraction is SWAR for bytes and halfwords.  Lane-contiguous accesses,
// DE_V vectors per thread with every load issued first.
constexpr int DE_V = 4;

template <int ES>
MC_DEV uint32_t swar_sub(uint32_t a, uint32_t b) {
  if constexpr (ES == 1) {
    constexpr uint32_t H = 0x80808080u;
    return ((a | H) - (b & ~H)) ^ ((a ^ ~b) & H);
  } else if constexpr (ES == 2) {
    constexpr uint32_t H = 0x80008000u;
    return ((a | H) - (b & ~H)) ^ ((a ^ ~b) & H);
  } else {
    return a - b;
  }
}

template <int ES, bool FL = false>
MC_DEV mc_u32x4 delta_vec(mc_u32x4 x, uint32_t p_lo, uint32_t p_hi) {
  // p_hi:p_lo = the 8 bytes just before x (p_hi the dword right before x.x)
  if constexpr (FL && ES == 8) {  // f8: IEEE double differences (numpy's f8 subtract)
    const double a0 = mc_bits_f64(((uint64_t)x.y << 32) | x.x), a1 = mc_bits_f64(((uint64_t)x.w << 32) | x.z);
    const double b0 = mc_bits_f64(((uint64_t)p_hi << 32) | p_lo);
    const uint64_t r0 = mc_f64_bits(mc_x86_nan(a0, b0, a0 - b0)), r1 = mc_f64_bits(mc_x86_nan(a1, a0, a1 - a0));
    return mc_u32x4{(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
  } else if constexpr (FL) {  // f4: IEEE float differences
    static_assert(ES == 4, "float same-type Delta encode: f4 / f8");
    const float a0 = mc_bits_f32(x.x), a1 = mc_bits_f32(x.y), a2 = mc_bits_f32(x.z), a3 = mc_bits_f32(x.w);
    const float b0 = mc_bits_f32(p_hi);
    return mc_u32x4{mc_f32_bits(mc_x86_nan(a0, b0, a0 - b0)), mc_f32_bits(mc_x86_nan(a1, a0, a1 - a0)),
                    mc_f32_bits(mc_x86_nan(a2, a1, a2 - a1)), mc_f32_bits(mc_x86_nan(a3, a2, a3 - a2))};
  } else if constexpr (ES == 8) {
    const uint64_t a0 = ((uint64_t)x.y << 32) | x.x, a1 = ((uint64_t)x.w << 32) | x.z;
    const uint64_t b0 = ((uint64_t)p_hi << 32) | p_lo;
    const uint64_t r0 = a0 - b0, r1 = a1 - a0;
    return mc_u32x4{(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
  } else if constexpr (ES == 4) {
    return mc_u32x4{x.x - p_hi, x.y - x.x, x.z - x.y, x.w - x.z};
  } else {
    constexpr uint32_t SH = 32 - 8 * ES;  // ({hi, lo} >> SH) = hi << 8ES | lo's top ES bytes
    const uint32_t s0 = __builtin_amdgcn_alignbit(x.x, p_hi, SH);
    const uint32_t s1 = __builtin_amdgcn_alignbit(x.y, x.x, SH);
    const uint32_t s2 = __builtin_amdgcn_alignbit(x.z, x.y, SH);
    const uint32_t s3 = __builtin_amdgcn_alignbit(x.w, x.z, SH);
    return mc_u32x4{swar_sub<ES>(x.x, s0), swar_sub<ES>(x.y, s1), swar_sub<ES>(x.z, s2),
                    swar_sub<ES>(x.w, s3)};
  }
}

// SW: bit 0 = the input is big-endian, bit 1 = the output is (the bytes of
// each element reversed after the load / before the store, v_perm_b32).
// FL: f4 / f8 (float differences; the first element is copied as it is).
// NV: 16-B vectors per thread (mc_sched.delta_enc_dv: DE_V or 2 x DE_V)
template <int ES, int SW = 0, bool FL = false, int NV = DE_V>
__global__ __launch_bounds__(MC_BLOCK) void k_delta_enc_same(const uint8_t *__restrict__ src,
                                                             uint8_t *__restrict__ dst, size_t nbytes,
                                                             size_t src_stride, size_t dst_stride) {
  constexpr int DE_V = NV;
  src += (size_t)blockIdx.y * src_stride;  // chunk blockIdx.y of a batch
  dst += (size_t)blockIdx.y * dst_stride;
  const int lane = threadIdx.x & 63;
  const size_t tb = (size_t)blockIdx.x * DE_V * 16 * MC_BLOCK;
  mc_u32x4 x[DE_V];
  uint32_t q_lo[DE_V], q_hi[DE_V];  // lane 0: the 8 bytes before its vector
#pragma unroll
  for (int r = 0; r < DE_V; ++r) {
    const size_t off = tb + (size_t)r * 16 * MC_BLOCK + 16 * (size_t)threadIdx.x;
    if (off + 16 <= nbytes) {
      x[r] = mc_ld16<true>(src + off);
    } else {
      uint32_t w[4] = {0, 0, 0, 0};
      for (int j = 0; j < 16 && off + j < nbytes; ++j) w[j >> 2] |= (uint32_t)src[off + j] << (8 * (j & 3));
      x[r] = mc_u32x4{w[0], w[1], w[2], w[3]};
    }
    q_lo[r] = q_hi[r] = 0;
    if (lane == 0 && off < nbytes && off > 0) {
      q_hi[r] = *reinterpret_cast<const uint32_t *>(src + off - 4);
      if (ES == 8) q_lo[r] = *reinterpret_cast<const uint32_t *>(src + off - 8);
    }
  }
  // the byte swaps of a big-endian input only after every load is issued: a
  // swap between them (the lane-0 loads are branches) waited for each load
  // before the next was issued (7 % slower than little-endian)
#pragma unroll
  for (int r = 0; r < DE_V; ++r) {
    const size_t off = tb + (size_t)r * 16 * MC_BLOCK + 16 * (size_t)threadIdx.x;
    if constexpr (SW & 1) {  // big-endian input: every element to register order
      x[r] = mc_bswap_vec<ES>(x[r]);
      const mc_u32x4 q = mc_bswap_vec<ES>(mc_u32x4{q_lo[r], q_hi[r], 0u, 0u});
      q_lo[r] = q.x;
      q_hi[r] = q.y;
    }
    // the previous 8 bytes: lane - 1's last dwords, lane 0's read above
    const uint32_t p_hi = mc_wave_shr1(x[r].w, q_hi[r]), p_lo = mc_wave_shr1(x[r].z, q_lo[r]);
    mc_u32x4 y = delta_vec<ES, FL>(x[r], p_lo, p_hi);
    if (FL && off == 0) {  // element 0 is stored as itself (x - 0 would turn -0.0 into +0.0)
      y.x = x[r].x;
      if constexpr (ES == 8) y.y = x[r].y;
    }
    if constexpr ((SW & 2) != 0) y = mc_bswap_vec<ES>(y);  // big-endian output
    if (off + 16 <= nbytes) {
      mc_st16<true>(dst + off, y);
    } else if (off < nbytes) {
      const uint32_t w[4] = {y.x, y.y, y.z, y.w};
      for (int j = 0; j < 16 && off + j < nbytes; ++j) dst[off + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
  }
}

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
static bool aligned_for(const void *p, int itemsize) {
  return ((uintptr_t)p % (uintptr_t)(4 * itemsize)) == 0;
}

static unsigned blocks_for(size_t n) {
  return (unsigned)((n + ELEMS_PER_BLOCK - 1) / ELEMS_PER_BLOCK);
}

// one constant-dtype instantiation per byte-order combination of the input
// (D) and output (A) dtypes: the byte reversals fold into the loads/stores
template <int KIND, int D, int T1, int T2, int A, int EPL = 4>
static void launch_map_bo(bool sd, bool sa, unsigned grid, const uint8_t *s, uint8_t *d, size_t n,
                          const MapParams &p, hipStream_t st) {
  constexpr int BE = MC_BIG_ENDIAN;
  if (!sd && !sa) k_map<KIND, D, T1, T2, A, true, EPL><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
  else if (sd && !sa) k_map<KIND, D | BE, T1, T2, A, true, EPL><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
  else if (!sd) k_map<KIND, D, T1, T2, A | BE, true, EPL><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
  else k_map<KIND, D | BE, T1, T2, A | BE, true, EPL><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
}

template <int KIND>
static int launch_map(const void *src, void *dst, size_t n, const MapParams &p, hipStream_t st) {
  if (n == 0) return MC_OK;
  if (!src || !dst) return MC_EINVAL;
  // input / output dtypes may be big-endian; the compute dtypes never are
  if (!mc_valid_dtype(p.d) || !mc_valid_native_dtype(p.t1) || !mc_valid_native_dtype(p.t2) ||
      !mc_valid_dtype(p.a))
    return MC_EINVAL;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  const bool vec = aligned_for(src, mc_itemsize(p.d)) && aligned_for(dst, mc_itemsize(p.a));
  const unsigned grid = blocks_for(n);
  const int db = mc_dt_base(p.d), ab = mc_dt_base(p.a);
  const bool sd = mc_dt_swapped(p.d), sa = mc_dt_swapped(p.a);
  // specialised hot paths (constant dtypes, any byte order): C4's FSO f4 -> i2
  // and i2 -> f4, Quantize and AsType between f4 and f8
  if (KIND == K_FSO_ENC && vec && db == MC_F4 && p.t1 == MC_F4 && p.t2 == MC_F4 && ab == MC_I2) {
    launch_map_bo<KIND, MC_F4, MC_F4, MC_F4, MC_I2>(sd, sa, grid, s, d, n, p, st);
  } else if (KIND == K_FSO_DEC && vec && db == MC_I2 && p.t1 == MC_F8 && p.t2 == MC_F8 && ab == MC_F4) {
    launch_map_bo<KIND, MC_I2, MC_F8, MC_F8, MC_F4>(sd, sa, grid, s, d, n, p, st);
  } else if (KIND == K_QUANTIZE && vec && db == MC_F4 && ab == MC_F4) {
    launch_map_bo<KIND, MC_F4, MC_F4, MC_F4, MC_F4>(sd, sa, grid, s, d, n, p, st);
  } else if (KIND == K_CAST && vec && db == MC_F4 && ab == MC_F8) {  // AsType / Quantize decode
    launch_map_bo<KIND, MC_F4, MC_F4, MC_F4, MC_F8, 2>(sd, sa, grid, s, d, n, p, st);
  } else if (KIND == K_CAST && vec && db == MC_F8 && ab == MC_F4) {
    launch_map_bo<KIND, MC_F8, MC_F8, MC_F8, MC_F4, 2>(sd, sa, grid, s, d, n, p, st);
  } else if (KIND == K_CAST && vec && db == MC_F4 && ab == MC_F4) {  // byte order only
    launch_map_bo<KIND, MC_F4, MC_F4, MC_F4, MC_F4>(sd, sa, grid, s, d, n, p, st);
  } else if (KIND == K_QUANTIZE && vec && db == MC_F8 && ab == MC_F4) {
    launch_map_bo<KIND, MC_F8, MC_F8, MC_F8, MC_F4, 2>(sd, sa, grid, s, d, n, p, st);
  } else if (vec && (mc_itemsize(p.d) == 8 || mc_itemsize(p.a) == 8)) {
    k_map<KIND, -1, -1, -1, -1, true, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
  } else if (vec) {
    k_map<KIND, -1, -1, -1, -1, true><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
  } else {
    k_map<KIND, -1, -1, -1, -1, false><<<grid, MC_BLOCK, 0, st>>>(s, d, n, p);
  }
  return mc_last_launch();
}

static McNum num_scalar(int dt, double f, int64_t i) {
  McNum r;
  r.f = mc_is_float(dt) ? f : 0.0;
  r.i = mc_is_float(dt) ? 0 : i;
  return r;
}

template <int ES, bool FL, int NV>
static void launch_delta_same_nv(int sw, dim3 g, const uint8_t *s, uint8_t *d, size_t nbytes, size_t ss, size_t ds,
                                 hipStream_t st) {
  g.x = (unsigned)((nbytes + (size_t)NV * 16 * MC_BLOCK - 1) / ((size_t)NV * 16 * MC_BLOCK));
  switch (sw) {
    case 0: k_delta_enc_same<ES, 0, FL, NV><<<g, MC_BLOCK, 0, st>>>(s, d, nbytes, ss, ds); break;
    case 1: k_delta_enc_same<ES, 1, FL, NV><<<g, MC_BLOCK, 0, st>>>(s, d, nbytes, ss, ds); break;
    case 2: k_delta_enc_same<ES, 2, FL, NV><<<g, MC_BLOCK, 0, st>>>(s, d, nbytes, ss, ds); break;
    default: k_delta_enc_same<ES, 3, FL, NV><<<g, MC_BLOCK, 0, st>>>(s, d, nbytes, ss, ds); break;
  }
}
// g.y = the batch rows; g.x follows from nbytes and the vectors per thread
template <int ES, bool FL = false>
static void launch_delta_same(int sw, dim3 g, const uint8_t *s, uint8_t *d, size_t nbytes, size_t ss, size_t ds,
                              hipStream_t st) {
  if (mc_sched.delta_enc_dv == 2 * DE_V) launch_delta_same_nv<ES, FL, 2 * DE_V>(sw, g, s, d, nbytes, ss, ds, st);
  else launch_delta_same_nv<ES, FL, DE_V>(sw, g, s, d, nbytes, ss, ds, st);
}

}  // namespace

extern "C" {

int mc_bitround(const void *src, void *dst, size_t n, int itemsize, int keepbits,
                mc_stream_t stream) {
  if (!(itemsize == 2 || itemsize == 4 || itemsize == 8)) return MC_EINVAL;
  const int mbits = itemsize == 2 ? 10 : itemsize == 4 ? 23 : 52;
  if (keepbits < 0 || keepbits > mbits) return MC_EINVAL;
  if (n == 0) return MC_OK;
  if (!src || !dst) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const size_t nbytes = n * (size_t)itemsize;
  if (keepbits == mbits) return mc_copy_rows_impl(src, nbytes, dst, nbytes, nbytes, 1, st);
  const McBitRound br = mc_make_bitround(itemsize, keepbits);
  const bool vec = ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  const size_t per = 16 * STEPS * MC_BLOCK;
  const unsigned grid = (unsigned)((nbytes + per - 1) / per);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  switch (itemsize) {
    case 2: k_bitround<2><<<grid, MC_BLOCK, 0, st>>>(s, d, nbytes, br, vec); break;
    case 4: k_bitround<4><<<grid, MC_BLOCK, 0, st>>>(s, d, nbytes, br, vec); break;
    default: k_bitround<8><<<grid, MC_BLOCK, 0, st>>>(s, d, nbytes, br, vec); break;
  }
  return mc_last_launch();
}

int mc_cast(const void *src, void *dst, size_t n, int from_dtype, int to_dtype,
            mc_stream_t stream) {
  // extended dtypes, and casts that only change byte order (a pure byte
  // reversal: the value kernel's float -> double -> float round trip would
  // quiet signalling NaNs, which numpy's byte-swapping cast keeps)
  if (mc_ext_code(from_dtype) || mc_ext_code(to_dtype) ||
      (mc_valid_dtype(from_dtype) && mc_valid_dtype(to_dtype) && mc_dt_base(from_dtype) == mc_dt_base(to_dtype)))
    return mc_cast_units(src, dst, n, from_dtype, to_dtype, 1, 1, stream);
  // compute dtypes are native: the byte order lives in the input/output codes
  const int fb = mc_dt_base(from_dtype);
  MapParams p{from_dtype, fb, fb, to_dtype, McNum{0, 0}, McNum{0, 0}};
  return launch_map<K_CAST>(src, dst, n, p, (hipStream_t)stream);
}

int mc_fso_encode(const void *src, void *dst, size_t n, int dtype, int t1, int t2, int astype,
                  double offset_f, int64_t offset_i, double scale_f, int64_t scale_i,
                  mc_stream_t stream) {
  if (mc_ext_code(dtype) || mc_ext_code(t1) || mc_ext_code(t2) || mc_ext_code(astype))
    return mc_fso_encode_x(src, dst, n, dtype, t1, t2, astype, offset_f, 0.0, offset_i, scale_f, 0.0, scale_i,
                           stream);
  MapParams p{dtype, t1, t2, astype, num_scalar(t1, offset_f, offset_i),
              num_scalar(t2, scale_f, scale_i)};
  return launch_map<K_FSO_ENC>(src, dst, n, p, (hipStream_t)stream);
}

int mc_fso_decode(const void *src, void *dst, size_t n, int astype, int t3, int t4, int dtype,
                  double scale, double offset, mc_stream_t stream) {
  if (mc_ext_code(dtype) || mc_ext_code(t3) || mc_ext_code(t4) || mc_ext_code(astype))
    return mc_fso_decode_x(src, dst, n, astype, t3, t4, dtype, scale, 0.0, offset, 0.0, stream);
  if (!mc_is_float(t3) || !mc_is_float(t4)) return MC_EINVAL;
  MapParams p{astype, t3, t4, dtype, num_scalar(t3, scale, 0), num_scalar(t4, offset, 0)};
  // integer inputs (exact in f64) divided in f64 by the constant scale
  if (t3 == MC_F8 && !mc_is_float(astype) && astype != MC_B1) {
    p.rcp = 1.0 / scale;
    p.fastdiv = mc_fastdiv_ok(scale);
  }
  return launch_map<K_FSO_DEC>(src, dst, n, p, (hipStream_t)stream);
}

int mc_quantize(const void *src, void *dst, size_t n, int dtype, int astype, double scale,
                mc_stream_t stream) {
  const auto ld = [](int t) { return mc_dt_base(t) == MC_F16L && mc_ext_code(t); };
  if ((ld(dtype) || mc_is_float(dtype)) && (ld(astype) || mc_is_float(astype)) && (ld(dtype) || ld(astype)))
    return mc_ext_quantize(src, dst, n, dtype, astype, scale, (hipStream_t)stream);
  if (!mc_is_float(dtype) || !mc_is_float(astype)) return MC_EINVAL;
  const int db = mc_dt_base(dtype);  // the computation's dtype (native)
  MapParams p{dtype, db, db, astype, num_scalar(dtype, scale, 0), McNum{0, 0}};
  return launch_map<K_QUANTIZE>(src, dst, n, p, (hipStream_t)stream);
}

// mc_sched.delta_enc_vec = 0 keeps same-width integer encodes on k_delta_enc
// (lab A/B only)
static bool delta_enc_vec_enabled() { return mc_sched.delta_enc_vec != 0; }

int mc_delta_encode(const void *src, void *dst, size_t n, int dtype, int astype,
                    mc_stream_t stream) {
  return mc_delta_encode_batch(src, 0, dst, 0, 1, n, dtype, astype, stream);
}

int mc_delta_encode_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                          size_t nchunks, size_t n, int dtype, int astype, mc_stream_t stream) {
  if (mc_ext_code(dtype) || mc_ext_code(astype))  // extended dtypes: single chunks only
    return nchunks == 1 ? mc_ext_delta_encode(src, dst, n, dtype, astype, (hipStream_t)stream)
                        : (nchunks == 0 ? MC_OK : MC_EINVAL);
  if (!mc_valid_dtype(dtype) || !mc_valid_dtype(astype)) return MC_EINVAL;
  if (n == 0 || nchunks == 0) return MC_OK;
  if (!src || !dst) return MC_EINVAL;
  const int ss = mc_itemsize(dtype), ds = mc_itemsize(astype);
  if (nchunks > 1 && (src_stride < n * ss || dst_stride < n * ds)) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  const bool vec = aligned_for(src, ss) && aligned_for(dst, ds) &&
                   (nchunks == 1 || (src_stride % (4 * ss) == 0 && dst_stride % (4 * ds) == 0));
  const bool al16 = (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0 &&
                    (nchunks == 1 || (src_stride % 16 == 0 && dst_stride % 16 == 0));
  constexpr size_t YMAX = 65535;
  for (size_t c0 = 0; c0 < nchunks; c0 += YMAX) {
    const dim3 grid(blocks_for(n), (unsigned)min(YMAX, nchunks - c0));
    const uint8_t *sc = s + c0 * src_stride;
    uint8_t *dc = d + c0 * dst_stride;
    // same-width integers: wrapping differences have the same bits whatever
    // the signedness, so every such pair runs the signed instantiation; the
    // constant-dtype k_delta_enc paths below are little-endian only (sw == 0)
    const int db = mc_dt_base(dtype), ab = mc_dt_base(astype);
    const int sw = (mc_dt_swapped(dtype) ? 1 : 0) | (mc_dt_swapped(astype) ? 2 : 0);
    const int same = (db == ab && db != MC_B1 && !mc_is_float(db)) ? ss : 0;
    if (al16 && db == ab && (db == MC_F4 || db == MC_F8)) {  // float same-type: IEEE differences
      const size_t per = (size_t)DE_V * 16 * MC_BLOCK;
      const dim3 g2((unsigned)((n * ss + per - 1) / per), grid.y);
      if (db == MC_F4) launch_delta_same<4, true>(sw, g2, sc, dc, n * 4, src_stride, dst_stride, st);
      else launch_delta_same<8, true>(sw, g2, sc, dc, n * 8, src_stride, dst_stride, st);
    } else if (same && al16 && delta_enc_vec_enabled()) {
      const size_t per = (size_t)DE_V * 16 * MC_BLOCK;
      const dim3 g2((unsigned)((n * ss + per - 1) / per), grid.y);
      if (same == 1) launch_delta_same<1>(0, g2, sc, dc, n, src_stride, dst_stride, st);
      else if (same == 2) launch_delta_same<2>(sw, g2, sc, dc, n * 2, src_stride, dst_stride, st);
      else if (same == 4) launch_delta_same<4>(sw, g2, sc, dc, n * 4, src_stride, dst_stride, st);
      else launch_delta_same<8>(sw, g2, sc, dc, n * 8, src_stride, dst_stride, st);
    } else if (sw) {
      if (vec) k_delta_enc<-1, -1, true><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, dtype, astype, src_stride, dst_stride);
      else k_delta_enc<-1, -1, false><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, dtype, astype, src_stride, dst_stride);
    } else if (vec && same == 1)
      k_delta_enc<MC_I1, MC_I1, true><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, MC_I1, MC_I1, src_stride, dst_stride);
    else if (vec && same == 2)
      k_delta_enc<MC_I2, MC_I2, true><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, MC_I2, MC_I2, src_stride, dst_stride);
    else if (vec && same == 4)
      k_delta_enc<MC_I4, MC_I4, true><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, MC_I4, MC_I4, src_stride, dst_stride);
    else if (vec && same == 8)
      k_delta_enc<MC_I8, MC_I8, true><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, MC_I8, MC_I8, src_stride, dst_stride);
    else if (vec)
      k_delta_enc<-1, -1, true><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, dtype, astype, src_stride, dst_stride);
    else
      k_delta_enc<-1, -1, false><<<grid, MC_BLOCK, 0, st>>>(sc, dc, n, dtype, astype, src_stride, dst_stride);
  }
  return mc_last_launch();
}

}  // extern "C"
