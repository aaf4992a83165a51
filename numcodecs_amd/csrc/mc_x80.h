// mc_x80.h -- numpy's longdouble ('<f16') arithmetic as gfx950 integer code.
//
// On x86-64 Linux (the reference's platform: numpy's npy_longdouble is the
// C `long double`) a longdouble is the x87 80-bit extended format stored in
// 16 bytes: a 64-bit significand with an explicit integer bit J (bytes 0-7),
// sign and 15-bit biased exponent (bytes 8-9) and 6 padding bytes that numpy
// leaves as whatever the output buffer held.  numpy's longdouble ufunc loops
// (umath loops.c.src: add/subtract/multiply/divide, rint = rintl) and casts
// (lowlevel_strided_loops.c.src: `(npy_double)x`, `(npy_int)x`, ...) compile
// to x87 instructions running at 64-bit precision with round-to-nearest-even,
// so every operation here is ONE correctly rounded x87 operation:
//   * operands in the formats x87 rejects (unnormals: J = 0 with a nonzero
//     exponent; pseudo-infinities / pseudo-NaNs: J = 0 with exponent 0x7fff)
//     raise invalid and give the "real indefinite" QNaN (sign 1, J and the
//     quiet bit set); pseudo-denormals (exponent 0, J = 1) are valid;
//   * NaN operands follow the x87 rules of the Intel SDM (vol. 1 table 4-7),
//     not SSE's first-operand rule: a QNaN beats an SNaN, between two NaNs of
//     the same kind the larger significand wins, SNaNs come out quieted;
//     x - y never flips the sign of a NaN y;
//   * gradual underflow (denormal results rounded on the denormal grid),
//     overflow to infinity;
//   * casts to float32/float64 round once (fst m32/m64); to float16 through
//     float32 (numpy's npy_float_to_half((float)x)); to integers truncate
//     (fistp with truncation, as gcc compiles the C casts): out of range / NaN
//     give the "integer indefinite" of the store width (int16 stores for i2
//     and, truncated, i1/u1; int32 for i4 and, truncated, u2; int64 for i8
//     and, truncated, u4; u8 as gcc's x >= 2^63 ? (x - 2^63) ^ 2^63 split).
// tests/test_x80.py checks every function against numpy on the host (this
// header compiled for the host, tests/native/x80_host.hip) on random and
// special operands; the device kernels run the same code.
#pragma once

#include "mc_common.h"

#define MC_X80_FN MC_HD

struct X80 {
  uint64_t m;   // significand, J = bit 63
  uint32_t se;  // sign << 15 | biased exponent (bias 16383)
};

typedef unsigned __int128 x80_u128;

enum X80Class { X80_ZERO = 0, X80_FINITE = 1, X80_INF = 2, X80_QNAN = 3, X80_SNAN = 4, X80_BAD = 5 };

constexpr int X80_BIAS = 16383;
constexpr uint64_t X80_J = 1ull << 63;
constexpr uint64_t X80_QUIET = 1ull << 62;

MC_X80_FN X80 x80_make(uint64_t m, uint32_t se) {
  X80 r;
  r.m = m;
  r.se = se & 0xffffu;
  return r;
}
MC_X80_FN X80 x80_indefinite() { return x80_make(X80_J | X80_QUIET, 0xffffu); }
MC_X80_FN X80 x80_inf(uint32_t s) { return x80_make(X80_J, (s << 15) | 0x7fffu); }
MC_X80_FN X80 x80_zero(uint32_t s) { return x80_make(0, s << 15); }
MC_X80_FN uint32_t x80_sign(X80 a) { return (a.se >> 15) & 1u; }
MC_X80_FN int x80_bexp(X80 a) { return (int)(a.se & 0x7fffu); }

MC_X80_FN int x80_class(X80 a) {
  const int e = x80_bexp(a);
  const bool j = (a.m >> 63) != 0;
  if (e == 0x7fff) {
    if (!j) return X80_BAD;  // pseudo-infinity / pseudo-NaN
    if ((a.m << 1) == 0) return X80_INF;
    return (a.m & X80_QUIET) ? X80_QNAN : X80_SNAN;
  }
  if (e == 0) return a.m == 0 ? X80_ZERO : X80_FINITE;  // denormal / pseudo-denormal
  return j ? X80_FINITE : X80_BAD;                       // unnormal
}
MC_X80_FN bool x80_is_nan_class(int c) { return c == X80_QNAN || c == X80_SNAN; }

MC_X80_FN int x80_clz64(uint64_t v) { return v ? __builtin_clzll(v) : 64; }
MC_X80_FN int x80_clz128(x80_u128 v) {
  const uint64_t hi = (uint64_t)(v >> 64);
  return hi ? __builtin_clzll(hi) : 64 + x80_clz64((uint64_t)v);
}

// The NaN result of a two-operand x87 operation with at least one NaN
// operand (a and b as the instruction sees them; neither of a format x87
// rejects).
MC_X80_FN X80 x80_nan2(X80 a, int ca, X80 b, int cb) {
  const bool an = x80_is_nan_class(ca), bn = x80_is_nan_class(cb);
  X80 r;
  if (an && bn) {
    if (ca != cb) {
      r = ca == X80_QNAN ? a : b;  // a QNaN beats an SNaN
    } else if (a.m != b.m) {
      r = a.m > b.m ? a : b;  // the larger significand
    } else {
      r = x80_sign(a) ? b : a;  // equal significands: the positive one
    }
  } else {
    r = an ? a : b;
  }
  r.m |= X80_QUIET;
  return r;
}

// value = R * 2^(E - X80_BIAS - 127) (R != 0), rounded to nearest even into
// the 80-bit format (gradual underflow, overflow to infinity)
MC_X80_FN X80 x80_round_pack(uint32_t s, x80_u128 R, int E) {
  const int k = x80_clz128(R);
  R <<= k;
  E -= k;
  if (E >= 0x7fff) return x80_inf(s);
  if (E <= 0) {
    const int sh = 1 - E;
    if (sh >= 128) {
      R = 1;  // sticky only
    } else {
      const x80_u128 lost = R & ((((x80_u128)1) << sh) - 1);
      R = (R >> sh) | (lost != 0 ? 1 : 0);
    }
    E = 0;
  }
  uint64_t m = (uint64_t)(R >> 64);
  const uint64_t rest = (uint64_t)R;
  const bool rnd = (rest >> 63) != 0, sticky = (rest << 1) != 0;
  if (rnd && (sticky || (m & 1))) {
    ++m;
    if (m == 0) {
      m = X80_J;
      ++E;
      if (E >= 0x7fff) return x80_inf(s);
    } else if (E == 0 && (m >> 63)) {
      E = 1;  // a denormal rounded up to the smallest normal
    }
  }
  if (m == 0) return x80_zero(s);
  return x80_make(m, (s << 15) | (uint32_t)E);
}

// exponent used for arithmetic: denormals and pseudo-denormals count as 1
MC_X80_FN int x80_eexp(X80 a) {
  const int e = x80_bexp(a);
  return e == 0 ? 1 : e;
}

// a + (negate_b ? -b : b)
MC_X80_FN X80 x80_addsub(X80 a, X80 b, bool negate_b) {
  // fast path: both operands normal (J set, exponent 1 .. 0x7ffe), exponent
  // gap <= 63 or > 65, normal result -- the running sums of a Delta decode
  // almost always; everything else takes the general code below (the same
  // results: tests/test_x80.py)
  {
    const uint32_t ea0 = a.se & 0x7fffu, eb0 = b.se & 0x7fffu;
    if (ea0 - 1u < 0x7ffeu && eb0 - 1u < 0x7ffeu && (a.m >> 63) && (b.m >> 63)) {
      uint32_t s1 = x80_sign(a), s2 = x80_sign(b) ^ (negate_b ? 1u : 0u);
      uint32_t e1 = ea0, e2 = eb0;
      uint64_t m1 = a.m, m2 = b.m;
      if (e1 < e2 || (e1 == e2 && m1 < m2)) {
        const uint32_t te = e1; e1 = e2; e2 = te;
        const uint64_t tm = m1; m1 = m2; m2 = tm;
        const uint32_t ts = s1; s1 = s2; s2 = ts;
      }
      const uint32_t d = e1 - e2;
      if (d > 65u) return x80_make(m1, (s1 << 15) | e1);  // |smaller| < half an ulp
      if (d <= 63u) {
        const uint64_t bh = m2 >> d, bl = d ? m2 << (64u - d) : 0;
        uint64_t hi, lo;
        int e = (int)e1;
        if (s1 == s2) {
          hi = m1 + bh;
          lo = bl;
          if (hi < m1) {  // carry out: shift the 129-bit sum right by one
            lo = (hi << 63) | (lo >> 1) | (lo & 1u);
            hi = X80_J | (hi >> 1);
            ++e;
          }
        } else {
          lo = 0 - bl;
          hi = m1 - bh - (bl != 0 ? 1u : 0u);
          if (hi == 0 && lo == 0) return x80_zero(0);
          const int k = hi ? x80_clz64(hi) : 64 + x80_clz64(lo);
          if (e - k < 1) goto general;  // a denormal result
          if (k >= 64) {
            hi = lo << (k - 64);
            lo = 0;
          } else if (k) {
            hi = (hi << k) | (lo >> (64 - k));
            lo <<= k;
          }
          e -= k;
        }
        if ((lo >> 63) && ((lo << 1) != 0 || (hi & 1u))) {
          if (++hi == 0) {
            hi = X80_J;
            ++e;
          }
        }
        if (e >= 0x7fff) return x80_inf(s1);
        return x80_make(hi, (s1 << 15) | (uint32_t)e);
      }
    }
  }
general:
  const int ca = x80_class(a), cb = x80_class(b);
  if (ca == X80_BAD || cb == X80_BAD) return x80_indefinite();
  if (x80_is_nan_class(ca) || x80_is_nan_class(cb)) return x80_nan2(a, ca, b, cb);
  const uint32_t sa = x80_sign(a), sb = x80_sign(b) ^ (negate_b ? 1u : 0u);
  if (ca == X80_INF || cb == X80_INF) {
    if (ca == X80_INF && cb == X80_INF) return sa == sb ? x80_inf(sa) : x80_indefinite();
    return ca == X80_INF ? x80_inf(sa) : x80_inf(sb);
  }
  if (ca == X80_ZERO && cb == X80_ZERO) return x80_zero(sa & sb);
  int ea = x80_eexp(a), eb = x80_eexp(b);
  uint64_t ma = a.m, mb = b.m;
  uint32_t s1 = sa, s2 = sb;
  if (ca == X80_ZERO) ea = 1;
  if (cb == X80_ZERO) eb = 1;
  if (ea < eb || (ea == eb && ma < mb)) {
    const int te = ea; ea = eb; eb = te;
    const uint64_t tm = ma; ma = mb; mb = tm;
    const uint32_t ts = s1; s1 = s2; s2 = ts;
  }
  const x80_u128 A = ((x80_u128)ma) << 62;
  x80_u128 B = ((x80_u128)mb) << 62;
  const int d = ea - eb;
  if (d >= 126) {
    B = mb != 0 ? 1 : 0;
  } else if (d > 0) {
    const x80_u128 lost = B & ((((x80_u128)1) << d) - 1);
    B = (B >> d) | (lost != 0 ? 1 : 0);
  }
  const x80_u128 R = s1 == s2 ? A + B : A - B;
  if (R == 0) return x80_zero(0);  // exact cancellation: +0 when rounding to nearest
  return x80_round_pack(s1, R, ea + 2);
}

MC_X80_FN X80 x80_add(X80 a, X80 b) { return x80_addsub(a, b, false); }
MC_X80_FN X80 x80_sub(X80 a, X80 b) { return x80_addsub(a, b, true); }

MC_X80_FN X80 x80_mul(X80 a, X80 b) {
  const int ca = x80_class(a), cb = x80_class(b);
  if (ca == X80_BAD || cb == X80_BAD) return x80_indefinite();
  if (x80_is_nan_class(ca) || x80_is_nan_class(cb)) return x80_nan2(a, ca, b, cb);
  const uint32_t s = x80_sign(a) ^ x80_sign(b);
  if (ca == X80_INF || cb == X80_INF) {
    if (ca == X80_ZERO || cb == X80_ZERO) return x80_indefinite();
    return x80_inf(s);
  }
  if (ca == X80_ZERO || cb == X80_ZERO) return x80_zero(s);
  const x80_u128 P = ((x80_u128)a.m) * b.m;
  return x80_round_pack(s, P, x80_eexp(a) + x80_eexp(b) - X80_BIAS + 1);
}

MC_X80_FN X80 x80_div(X80 a, X80 b) {
  const int ca = x80_class(a), cb = x80_class(b);
  if (ca == X80_BAD || cb == X80_BAD) return x80_indefinite();
  if (x80_is_nan_class(ca) || x80_is_nan_class(cb)) return x80_nan2(a, ca, b, cb);
  const uint32_t s = x80_sign(a) ^ x80_sign(b);
  if (ca == X80_INF) return cb == X80_INF ? x80_indefinite() : x80_inf(s);
  if (cb == X80_INF) return x80_zero(s);
  if (cb == X80_ZERO) return ca == X80_ZERO ? x80_indefinite() : x80_inf(s);
  if (ca == X80_ZERO) return x80_zero(s);
  // normalise both significands (denormals), then 67 quotient bits by
  // restoring division and a sticky bit from the remainder
  const int ka = x80_clz64(a.m), kb = x80_clz64(b.m);
  const uint64_t ma = a.m << ka, mb = b.m << kb;
  const int ea = x80_eexp(a) - ka, eb = x80_eexp(b) - kb;
  x80_u128 r = ma, q = 0;
  for (int i = 0; i < 67; ++i) {
    const bool bit = r >= (x80_u128)mb;
    if (bit) r -= mb;
    q = (q << 1) | (bit ? 1 : 0);
    r <<= 1;
  }
  const x80_u128 R = (q << 1) | (r != 0 ? 1 : 0);
  return x80_round_pack(s, R, ea - eb + X80_BIAS + 60);
}

// rintl: round to an integral value, ties to even (np.around / np.rint)
MC_X80_FN X80 x80_rint(X80 a) {
  const int c = x80_class(a);
  if (c == X80_BAD) return x80_indefinite();
  if (c == X80_QNAN || c == X80_SNAN) {
    a.m |= X80_QUIET;
    return a;
  }
  if (c == X80_INF || c == X80_ZERO) return a;
  const uint32_t s = x80_sign(a);
  const int e = x80_eexp(a);
  const int f = X80_BIAS + 63 - e;  // fraction bits in the significand
  if (f <= 0) return x80_round_pack(s, ((x80_u128)a.m) << 64, e);  // already integral (normalised)
  if (f > 64) return x80_zero(s);   // |a| < 0.5
  uint64_t ip, rem, half;
  if (f == 64) {
    ip = 0;
    rem = a.m;
    half = X80_J;
  } else {
    ip = a.m >> f;
    rem = a.m & ((1ull << f) - 1);
    half = 1ull << (f - 1);
  }
  if (rem > half || (rem == half && (ip & 1))) ++ip;
  if (ip == 0) return x80_zero(s);
  return x80_round_pack(s, ((x80_u128)ip) << 64, X80_BIAS + 63);
}

// ---------------------------------------------------------------------------
// conversions from the other numpy dtypes (exact; signalling NaNs quieted as
// x87 loads quiet them)
// ---------------------------------------------------------------------------
MC_X80_FN X80 x80_from_f64_bits(uint64_t b) {
  const uint32_t s = (uint32_t)(b >> 63);
  const int E = (int)((b >> 52) & 0x7ff);
  const uint64_t F = b & ((1ull << 52) - 1);
  if (E == 0x7ff) {
    if (F == 0) return x80_inf(s);
    return x80_make(X80_J | X80_QUIET | (F << 11), (s << 15) | 0x7fffu);
  }
  if (E == 0) {
    if (F == 0) return x80_zero(s);
    const int k = x80_clz64(F);
    return x80_make(F << k, (s << 15) | (uint32_t)(X80_BIAS + 63 - 1074 - k));
  }
  return x80_make(X80_J | (F << 11), (s << 15) | (uint32_t)(E - 1023 + X80_BIAS));
}

MC_X80_FN X80 x80_from_f32_bits(uint32_t b) {
  const uint32_t s = b >> 31;
  const int E = (int)((b >> 23) & 0xff);
  const uint64_t F = b & ((1u << 23) - 1);
  if (E == 0xff) {
    if (F == 0) return x80_inf(s);
    return x80_make(X80_J | X80_QUIET | (F << 40), (s << 15) | 0x7fffu);
  }
  if (E == 0) {
    if (F == 0) return x80_zero(s);
    const int k = x80_clz64(F);
    return x80_make(F << k, (s << 15) | (uint32_t)(X80_BIAS + 63 - 149 - k));
  }
  return x80_make(X80_J | (F << 40), (s << 15) | (uint32_t)(E - 127 + X80_BIAS));
}

MC_X80_FN X80 x80_from_u64(uint64_t v, uint32_t s = 0) {
  if (v == 0) return x80_zero(0);
  const int k = x80_clz64(v);
  return x80_make(v << k, (s << 15) | (uint32_t)(X80_BIAS + 63 - k));
}
MC_X80_FN X80 x80_from_i64(int64_t v) {
  return v < 0 ? x80_from_u64(0 - (uint64_t)v, 1) : x80_from_u64((uint64_t)v, 0);
}

// ---------------------------------------------------------------------------
// conversions to the other numpy dtypes
// ---------------------------------------------------------------------------
// round to an IEEE binary format of `p` significand bits (hidden bit
// included), exponent bias `bias` and all-ones exponent `emax_field`:
// returns the bit pattern (fst m32 / m64)
MC_X80_FN uint64_t x80_to_ieee(X80 a, int p, int bias, int emax_field) {
  const int c = x80_class(a);
  const int fbits = p - 1;
  const int signpos = p == 53 ? 63 : 31;
  const uint64_t s = (uint64_t)x80_sign(a) << signpos;
  const uint64_t expmask = (uint64_t)emax_field << fbits;
  // a rejected format: the default NaN of the destination (sign set, quiet)
  if (c == X80_BAD) return (1ull << signpos) | expmask | (1ull << (fbits - 1));
  if (c == X80_QNAN || c == X80_SNAN)
    return s | expmask | (1ull << (fbits - 1)) | ((a.m >> (64 - p)) & ((1ull << fbits) - 1));
  if (c == X80_INF) return s | expmask;
  if (c == X80_ZERO) return s;
  // value = m * 2^(e - bias80 - 63), m normalised to bit 63
  const int k = x80_clz64(a.m);
  const uint64_t m = a.m << k;
  const int E = x80_eexp(a) - X80_BIAS - k;  // unbiased exponent of the leading 1
  const int emin = 1 - bias;
  if (E > bias) return s | expmask;  // overflow
  int sh = 64 - p;  // bits dropped for a normal result
  int ef;           // biased exponent field before adding the significand
  if (E >= emin) {
    ef = E + bias - 1;  // the hidden bit of r adds the missing 1
  } else {
    sh += emin - E;
    ef = 0;
  }
  uint64_t r;
  bool rnd, sticky;
  if (sh >= 65) {
    r = 0;
    rnd = false;
    sticky = true;
  } else if (sh == 64) {
    r = 0;
    rnd = (m >> 63) != 0;
    sticky = (m << 1) != 0;
  } else {
    r = m >> sh;
    const uint64_t rest = m << (64 - sh);
    rnd = (rest >> 63) != 0;
    sticky = (rest << 1) != 0;
  }
  if (rnd && (sticky || (r & 1))) ++r;
  const uint64_t v = ((uint64_t)ef << fbits) + r;
  if ((v >> fbits) >= (uint64_t)emax_field) return s | expmask;  // overflow
  return s | v;
}
MC_X80_FN uint64_t x80_to_f64_bits(X80 a) { return x80_to_ieee(a, 53, 1023, 0x7ff); }
MC_X80_FN uint32_t x80_to_f32_bits(X80 a) { return (uint32_t)x80_to_ieee(a, 24, 127, 0xff); }

// truncation toward zero to a signed integer of `bits` (16/32/64), the
// integer indefinite (only the sign bit set) when out of range / NaN / inf /
// a rejected format
MC_X80_FN int64_t x80_trunc_int(X80 a, int bits) {
  const int c = x80_class(a);
  const int64_t indef = bits == 64 ? INT64_MIN : -(((int64_t)1) << (bits - 1));
  if (c == X80_ZERO) return 0;
  if (c != X80_FINITE) return indef;
  const int e = x80_eexp(a);
  const int f = X80_BIAS + 63 - e;
  if (f >= 64) return 0;
  if (f <= 0) return indef;  // |a| >= 2^63
  const uint64_t mag = a.m >> f;
  const bool neg = x80_sign(a) != 0;
  if (bits == 64) return neg ? (int64_t)(0 - mag) : (int64_t)mag;  // mag < 2^63
  const uint64_t lim = 1ull << (bits - 1);
  if (neg ? mag > lim : mag >= lim) return indef;
  return neg ? -(int64_t)mag : (int64_t)mag;
}

MC_X80_FN bool x80_ge_2p63(X80 a) {  // a >= 2^63 (false for NaN / rejected formats)
  const int c = x80_class(a);
  if (c == X80_INF) return x80_sign(a) == 0;
  if (c != X80_FINITE || x80_sign(a)) return false;
  return x80_eexp(a) >= X80_BIAS + 63;
}

MC_X80_FN uint64_t x80_to_u64(X80 a) {
  if (x80_ge_2p63(a)) {
    const X80 t = x80_sub(a, x80_make(X80_J, X80_BIAS + 63));
    return (uint64_t)x80_trunc_int(t, 64) ^ (1ull << 63);
  }
  return (uint64_t)x80_trunc_int(a, 64);
}

MC_X80_FN bool x80_nonzero(X80 a) { return x80_class(a) != X80_ZERO; }  // x != 0 (NaN: true)

// 16 storage bytes <-> X80 (little-endian: significand, then sign/exponent;
// the 6 padding bytes are written as zero)
MC_X80_FN X80 x80_from_words(uint64_t lo, uint64_t hi) { return x80_make(lo, (uint32_t)(hi & 0xffffu)); }

// ---------------------------------------------------------------------------
// numpy astype between longdouble and the other real dtypes, on raw element
// bits (little-endian storage value, byte order already normalised)
// ---------------------------------------------------------------------------
MC_X80_FN X80 x80_from_bits(uint64_t b, int dt) {
  switch (mc_dt_base(dt)) {
    case MC_B1: return x80_from_u64((b & 0xffu) != 0);
    case MC_I1: return x80_from_i64((int8_t)b);
    case MC_I2: return x80_from_i64((int16_t)b);
    case MC_I4: return x80_from_i64((int32_t)b);
    case MC_U1: return x80_from_u64((uint8_t)b);
    case MC_U2: return x80_from_u64((uint16_t)b);
    case MC_U4: return x80_from_u64((uint32_t)b);
    case MC_U8: return x80_from_u64(b);
    case MC_F2: return x80_from_f32_bits(mc_half_to_float_bits((uint16_t)b));  // (npy_longdouble)npy_half_to_float
    case MC_F4: return x80_from_f32_bits((uint32_t)b);
    case MC_F8: return x80_from_f64_bits(b);
    default: return x80_from_i64((int64_t)b);  // i8, timedelta64 / datetime64 ticks (NaT = INT64_MIN)
  }
}

MC_X80_FN uint64_t x80_to_bits(X80 a, int dt) {
  switch (mc_dt_base(dt)) {
    case MC_B1: return x80_nonzero(a) ? 1u : 0u;
    case MC_I1: return (uint8_t)x80_trunc_int(a, 16);
    case MC_U1: return (uint8_t)x80_trunc_int(a, 16);
    case MC_I2: return (uint16_t)x80_trunc_int(a, 16);
    case MC_U2: return (uint16_t)x80_trunc_int(a, 32);
    case MC_I4: return (uint32_t)x80_trunc_int(a, 32);
    case MC_U4: return (uint32_t)x80_trunc_int(a, 64);
    case MC_U8: return x80_to_u64(a);
    case MC_F2: return mc_float_bits_to_half(x80_to_f32_bits(a));  // npy_float_to_half((float)x)
    case MC_F4: return x80_to_f32_bits(a);
    case MC_F8: return x80_to_f64_bits(a);
    default: return (uint64_t)x80_trunc_int(a, 64);  // i8, timedelta64 / datetime64 ticks
  }
}
