// mc_num.h -- numpy-exact scalar arithmetic on device for the elementwise
// codecs (fixedscaleoffset.py, quantize.py, delta.py).
//
// A value of any numpy dtype is carried as McNum: floats in `f` (a double,
// which holds every f16/f32 value exactly), integers and bools in `i` (two's
// complement, sign- or zero-extended from the dtype's width).  Each operation
// takes the dtype it is computed in and rounds/wraps exactly as numpy's ufunc
// loop for that dtype does:
//   f64: IEEE double op;  f32: IEEE float op (the double carrier is exact, and
//   LLVM folds fptrunc(fpext(x)) so specialised kernels run pure f32 code);
//   f16: the op in float32, rounded to half (numpy's half loops);
//   integers: wrap-around in the dtype's width;  bool: numpy's bool loops.
// Casts follow numpy `astype` (unsafe) as compiled for x86-64 (mc_common.h).
// When a kernel is instantiated with constant dtypes every switch folds away.
#pragma once

#include "mc_common.h"

#include <stdlib.h>

struct McNum {
  double f;
  int64_t i;
};

MC_HD McNum mc_num_f(double f) { McNum r; r.f = f; r.i = 0; return r; }
MC_HD McNum mc_num_i(int64_t i) { McNum r; r.f = 0.0; r.i = i; return r; }

// wrap a 64-bit integer to dtype width (sign- or zero-extend back to 64 bits)
MC_DEV int64_t mc_wrap(int64_t v, int dt) {
  switch (mc_dt_base(dt)) {
    case MC_B1: return v != 0;
    case MC_I1: return (int64_t)(int8_t)v;
    case MC_I2: return (int64_t)(int16_t)v;
    case MC_I4: return (int64_t)(int32_t)v;
    case MC_U1: return (int64_t)(uint8_t)v;
    case MC_U2: return (int64_t)(uint16_t)v;
    case MC_U4: return (int64_t)(uint32_t)v;
    default: return v;  // I8, U8 (u8 kept as its bit pattern)
  }
}

// raw bits (low itemsize bytes, as loaded little-endian) -> value; a
// big-endian dtype's bytes are reversed first
MC_DEV McNum mc_num_from_bits(uint64_t b, int dt) {
  b = mc_to_storage(b, dt);
  switch (mc_dt_base(dt)) {
    case MC_F2: return mc_num_f((double)mc_half_to_float((uint16_t)b));
    case MC_F4: return mc_num_f((double)mc_bits_f32((uint32_t)b));
    case MC_F8: return mc_num_f(mc_bits_f64(b));
    case MC_B1: return mc_num_i((b & 0xffu) != 0);
    default: return mc_num_i(mc_wrap((int64_t)b, dt));
  }
}

// value (already in dt) -> raw bits as stored (big-endian dtypes reversed)
MC_DEV uint64_t mc_num_to_bits(McNum v, int dt) {
  uint64_t b;
  switch (mc_dt_base(dt)) {
    case MC_F2: b = mc_float_to_half((float)v.f); break;  // exact: v.f holds a half value
    case MC_F4: b = mc_f32_bits((float)v.f); break;
    case MC_F8: b = mc_f64_bits(v.f); break;
    default: b = (uint64_t)v.i; break;
  }
  return mc_to_storage(b, dt);
}

// numpy astype(from -> to) (byte order is storage only: ignored here)
MC_DEV McNum mc_num_cast(McNum v, int from, int to) {
  from = mc_dt_base(from);
  to = mc_dt_base(to);
  if (from == to) return v;
  const bool ff = mc_is_float(from), tf = mc_is_float(to);
  if (to == MC_B1) return mc_num_i(ff ? (v.f != 0.0) : (v.i != 0));
  if (ff && tf) {
    if (to == MC_F8) return v;                           // widening is exact
    if (to == MC_F4) return mc_num_f((double)(float)v.f);  // from f8: RNE
    // to f16: numpy converts double directly (npy_double_to_half), float via
    // npy_float_to_half
    const uint16_t h = from == MC_F8 ? mc_double_to_half(v.f) : mc_float_to_half((float)v.f);
    return mc_num_f((double)mc_half_to_float(h));
  }
  if (!ff && !tf) return mc_num_i(mc_wrap(v.i, to));
  if (ff) {  // float -> integer, x86-64 cvtt semantics then truncation
    const double x = v.f;
    switch (to) {
      case MC_I8: return mc_num_i(mc_cvtt_i64(x));
      case MC_U4: {
        // numpy's vectorised x86-64 loop (cvttpd2dq/cvttps2dq with the
        // 2^31 bias trick), which converts every element of a chunk except
        // the scalar remainder of the SIMD loop; numpy's scalar remainder
        // truncates a 64-bit conversion instead, so numpy itself is
        // position-dependent for |x| >= 2^32 ("casts").
        const uint32_t r = x >= 2147483648.0
                               ? ((uint32_t)mc_cvtt_i32(x - 2147483648.0) ^ 0x80000000u)
                               : (uint32_t)mc_cvtt_i32(x);
        return mc_num_i((int64_t)r);
      }
      case MC_U8: return mc_num_i((int64_t)mc_cvtt_u64(x));
      default: return mc_num_i(mc_wrap((int64_t)mc_cvtt_i32(x), to));
    }
  }
  // integer/bool -> float
  const bool is_u8 = from == MC_U8;
  switch (to) {
    case MC_F8:
      return mc_num_f(is_u8 ? (double)(uint64_t)v.i : (double)v.i);
    case MC_F4:
      return mc_num_f((double)(is_u8 ? (float)(uint64_t)v.i : (float)v.i));
    default: {  // f16 via float (numpy: npy_float_to_half((float)x))
      const float f = is_u8 ? (float)(uint64_t)v.i : (float)v.i;
      return mc_num_f((double)mc_half_to_float(mc_float_to_half(f)));
    }
  }
}

enum McOp { MC_OP_ADD, MC_OP_SUB, MC_OP_MUL, MC_OP_DIV };

// The NaN an x86-64 SSE add/sub/mul/div returns (numpy's float loops): the
// first operand's NaN quieted, else the second's, else -- an invalid
// operation such as inf - inf -- the negative "real indefinite" quiet NaN.
// The GPU computes x - y as x + (-y), which flips the sign of a NaN y, and
// its default NaN is positive; non-NaN results are the same IEEE values.
template <typename F>
MC_DEV F mc_x86_nan(F x, F y, F r) {
  if (!__builtin_isnan(r)) return r;
  if constexpr (sizeof(F) == 8) {
    constexpr uint64_t Q = 1ull << 51, DEF = 0xFFF8000000000000ull;
    const uint64_t b = __builtin_isnan(x) ? mc_f64_bits(x) | Q : __builtin_isnan(y) ? mc_f64_bits(y) | Q : DEF;
    return mc_bits_f64(b);
  } else {
    constexpr uint32_t Q = 1u << 22, DEF = 0xFFC00000u;
    const uint32_t b = __builtin_isnan(x) ? mc_f32_bits(x) | Q : __builtin_isnan(y) ? mc_f32_bits(y) | Q : DEF;
    return mc_bits_f32(b);
  }
}

// a <op> b with both operands already in dtype dt
MC_DEV McNum mc_num_binop(McNum a, McNum b, int op, int dt) {
  dt = mc_dt_base(dt);
  if (dt == MC_F8) {
    double r;
    switch (op) {
      case MC_OP_ADD: r = a.f + b.f; break;
      case MC_OP_SUB: r = a.f - b.f; break;
      case MC_OP_MUL: r = a.f * b.f; break;
      default: r = a.f / b.f; break;
    }
    return mc_num_f(mc_x86_nan(a.f, b.f, r));
  }
  if (dt == MC_F4 || dt == MC_F2) {
    const float x = (float)a.f, y = (float)b.f;
    float r;
    switch (op) {
      case MC_OP_ADD: r = x + y; break;
      case MC_OP_SUB: r = x - y; break;
      case MC_OP_MUL: r = x * y; break;
      default: r = x / y; break;
    }
    r = mc_x86_nan(x, y, r);
    if (dt == MC_F2) r = mc_half_to_float(mc_float_to_half(r));
    return mc_num_f((double)r);
  }
  if (dt == MC_B1) {  // numpy bool loops: add = or, sub = xor (diff), mul = and
    switch (op) {
      case MC_OP_ADD: return mc_num_i((a.i | b.i) != 0);
      case MC_OP_SUB: return mc_num_i((a.i != 0) != (b.i != 0));
      default: return mc_num_i((a.i & b.i) != 0);
    }
  }
  const uint64_t x = (uint64_t)a.i, y = (uint64_t)b.i;
  uint64_t r;
  switch (op) {
    case MC_OP_ADD: r = x + y; break;
    case MC_OP_SUB: r = x - y; break;
    default: r = x * y; break;  // integer true division never reaches here
  }
  return mc_num_i(mc_wrap((int64_t)r, dt));
}

// np.around(x) == np.rint for floats (round half to even); identity for ints
MC_DEV McNum mc_num_rint(McNum v, int dt) {
  dt = mc_dt_base(dt);
  if (dt == MC_F8) return mc_num_f(__builtin_rint(v.f));
  if (dt == MC_F4) return mc_num_f((double)__builtin_rintf((float)v.f));
  if (dt == MC_F2) {
    const float r = __builtin_rintf((float)v.f);
    return mc_num_f((double)mc_half_to_float(mc_float_to_half(r)));
  }
  return v;
}

// ---------------------------------------------------------------------------
// element I/O: 4 consecutive elements per lane per step
// ---------------------------------------------------------------------------
MC_DEV uint64_t mc_load_elem(const uint8_t *p, size_t idx, int size) {
  switch (size) {
    case 1: return p[idx];
    case 2: return reinterpret_cast<const uint16_t *>(p)[idx];
    case 4: return reinterpret_cast<const uint32_t *>(p)[idx];
    default: return reinterpret_cast<const uint64_t *>(p)[idx];
  }
}
MC_DEV void mc_store_elem(uint8_t *p, size_t idx, int size, uint64_t v) {
  switch (size) {
    case 1: p[idx] = (uint8_t)v; break;
    case 2: reinterpret_cast<uint16_t *>(p)[idx] = (uint16_t)v; break;
    case 4: reinterpret_cast<uint32_t *>(p)[idx] = (uint32_t)v; break;
    default: reinterpret_cast<uint64_t *>(p)[idx] = v; break;
  }
}
// byte-wise variants for unaligned buffers
MC_DEV uint64_t mc_load_elem_u(const uint8_t *p, size_t idx, int size) {
  uint64_t v = 0;
  for (int k = 0; k < size; ++k) v |= (uint64_t)p[idx * size + k] << (8 * k);
  return v;
}
MC_DEV void mc_store_elem_u(uint8_t *p, size_t idx, int size, uint64_t v) {
  for (int k = 0; k < size; ++k) p[idx * size + k] = (uint8_t)(v >> (8 * k));
}

// 4 consecutive elements (4*size bytes, 4*size-aligned) as one vector access
template <bool NT = false>
MC_DEV void mc_load4(const uint8_t *p, int size, uint64_t (&e)[4]) {
  switch (size) {
    case 1: {
      const uint32_t w = mc_ld4<NT>(p);
      for (int k = 0; k < 4; ++k) e[k] = (w >> (8 * k)) & 0xffu;
    } break;
    case 2: {
      const mc_u32x2 w = mc_ld8<NT>(p);
      e[0] = w.x & 0xffffu; e[1] = w.x >> 16; e[2] = w.y & 0xffffu; e[3] = w.y >> 16;
    } break;
    case 4: {
      const mc_u32x4 w = mc_ld16<NT>(p);
      e[0] = w.x; e[1] = w.y; e[2] = w.z; e[3] = w.w;
    } break;
    default: {
      const mc_u32x4 a = mc_ld16<NT>(p), b = mc_ld16<NT>(p + 16);
      e[0] = ((uint64_t)a.y << 32) | a.x; e[1] = ((uint64_t)a.w << 32) | a.z;
      e[2] = ((uint64_t)b.y << 32) | b.x; e[3] = ((uint64_t)b.w << 32) | b.z;
    } break;
  }
}
// 2 consecutive elements (2*size bytes, 2*size-aligned) as one vector access
template <bool NT = false>
MC_DEV void mc_load2(const uint8_t *p, int size, uint64_t (&e)[2]) {
  switch (size) {
    case 1: {
      const uint32_t w = *reinterpret_cast<const uint16_t *>(p);
      e[0] = w & 0xffu; e[1] = w >> 8;
    } break;
    case 2: {
      const uint32_t w = mc_ld4<NT>(p);
      e[0] = w & 0xffffu; e[1] = w >> 16;
    } break;
    case 4: {
      const mc_u32x2 w = mc_ld8<NT>(p);
      e[0] = w.x; e[1] = w.y;
    } break;
    default: {
      const mc_u32x4 a = mc_ld16<NT>(p);
      e[0] = ((uint64_t)a.y << 32) | a.x; e[1] = ((uint64_t)a.w << 32) | a.z;
    } break;
  }
}
template <bool NT = false>
MC_DEV void mc_store2(uint8_t *p, int size, const uint64_t (&e)[2]) {
  switch (size) {
    case 1: *reinterpret_cast<uint16_t *>(p) = (uint16_t)((e[0] & 0xff) | ((e[1] & 0xff) << 8)); break;
    case 2: mc_st4<NT>(p, (uint32_t)((e[0] & 0xffff) | ((e[1] & 0xffff) << 16))); break;
    case 4: mc_st8<NT>(p, mc_u32x2{(uint32_t)e[0], (uint32_t)e[1]}); break;
    default:
      mc_st16<NT>(p, mc_u32x4{(uint32_t)e[0], (uint32_t)(e[0] >> 32), (uint32_t)e[1], (uint32_t)(e[1] >> 32)});
      break;
  }
}

template <bool NT = false>
MC_DEV void mc_store4(uint8_t *p, int size, const uint64_t (&e)[4]) {
  switch (size) {
    case 1:
      mc_st4<NT>(p, (uint32_t)((e[0] & 0xff) | ((e[1] & 0xff) << 8) | ((e[2] & 0xff) << 16) |
                                  ((e[3] & 0xff) << 24)));
      break;
    case 2:
      mc_st8<NT>(p, mc_u32x2{(uint32_t)((e[0] & 0xffff) | ((e[1] & 0xffff) << 16)),
                                (uint32_t)((e[2] & 0xffff) | ((e[3] & 0xffff) << 16))});
      break;
    case 4:
      mc_st16<NT>(p, mc_u32x4{(uint32_t)e[0], (uint32_t)e[1], (uint32_t)e[2], (uint32_t)e[3]});
      break;
    default:
      mc_st16<NT>(p, mc_u32x4{(uint32_t)e[0], (uint32_t)(e[0] >> 32), (uint32_t)e[1],
                                 (uint32_t)(e[1] >> 32)});
      mc_st16<NT>(p + 16, mc_u32x4{(uint32_t)e[2], (uint32_t)(e[2] >> 32), (uint32_t)e[3],
                                      (uint32_t)(e[3] >> 32)});
      break;
  }
}

// Correctly rounded a / b for a constant b from rcp = RN(1/b) (Markstein):
// y = RN(a*rcp) is within an ulp of a/b, r = a - y*b is exact in one FMA,
// and RN(y + r*rcp) is RN(a/b).  Used only where the host has checked that
// a/b and r stay in the normal range (|b| in [2^-500, 2^500], |a| < 2^64);
// tests/test_gpu_c4.py compares it with IEEE division on every int16 for 15
// scales.  When r == 0, y is already the exact quotient (and keeps the sign
// of a zero).
MC_DEV double mc_div_by_const(double a, double b, double rcp) {
  const double y = a * rcp;
  const double r = __builtin_fma(-y, b, a);
  return r == 0.0 ? y : __builtin_fma(r, rcp, y);
}

// integer numerators (|a| < 2^64) divided by a scale in [2^-500, 2^500]: the
// quotient and the FMA residual stay normal, so mc_div_by_const is exact.
// mc_sched.fastdiv = 0 forces IEEE division (lab A/B and tests).
static inline bool mc_fastdiv_ok(double scale) {
  const double m = scale < 0 ? -scale : scale;
  return mc_sched.fastdiv != 0 && m >= 0x1p-500 && m <= 0x1p500;
}
