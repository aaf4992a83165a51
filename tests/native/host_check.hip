// host_check.hip -- numcodecs_amd/csrc/mc_x80.h (longdouble arithmetic) and
// mc_cal.h (calendar datetime casts) compiled for the HOST, so that
// tests/test_x80.py can compare the device kernels' scalar code with numpy's
// own results on the build machine (test infrastructure: nothing in the
// product loads this library).  Every function maps an operation over arrays
// (longdoubles as 16-byte little-endian elements).
#include "../../numcodecs_amd/csrc/mc_cal.h"
#include "../../numcodecs_amd/csrc/mc_x80.h"

#include <string.h>

namespace {
X80 ld_at(const uint8_t *p, size_t i) {
  uint64_t lo, hi = 0;
  memcpy(&lo, p + 16 * i, 8);
  memcpy(&hi, p + 16 * i + 8, 2);
  return x80_from_words(lo, hi);
}
void ld_put(uint8_t *p, size_t i, X80 v) {
  memset(p + 16 * i, 0, 16);
  memcpy(p + 16 * i, &v.m, 8);
  const uint16_t se = (uint16_t)v.se;
  memcpy(p + 16 * i + 8, &se, 2);
}
int dt_size(int dt) {
  switch (mc_dt_base(dt)) {
    case MC_B1: case MC_I1: case MC_U1: return 1;
    case MC_I2: case MC_U2: case MC_F2: return 2;
    case MC_I4: case MC_U4: case MC_F4: return 4;
    default: return 8;
  }
}
}  // namespace

extern "C" {

// op: 0 add, 1 sub, 2 mul, 3 div
int x80h_binop(int op, const void *a, const void *b, void *out, size_t n) {
  const uint8_t *pa = static_cast<const uint8_t *>(a), *pb = static_cast<const uint8_t *>(b);
  uint8_t *po = static_cast<uint8_t *>(out);
  for (size_t i = 0; i < n; ++i) {
    const X80 x = ld_at(pa, i), y = ld_at(pb, i);
    X80 r;
    switch (op) {
      case 0: r = x80_add(x, y); break;
      case 1: r = x80_sub(x, y); break;
      case 2: r = x80_mul(x, y); break;
      case 3: r = x80_div(x, y); break;
      default: return -1;
    }
    ld_put(po, i, r);
  }
  return 0;
}

int x80h_rint(const void *a, void *out, size_t n) {
  for (size_t i = 0; i < n; ++i) ld_put(static_cast<uint8_t *>(out), i, x80_rint(ld_at(static_cast<const uint8_t *>(a), i)));
  return 0;
}

// numpy astype(dt -> longdouble) of n elements of mc_dtype dt (native order)
int x80h_from(int dt, const void *src, void *out, size_t n) {
  const int es = dt_size(dt);
  for (size_t i = 0; i < n; ++i) {
    uint64_t b = 0;
    memcpy(&b, static_cast<const uint8_t *>(src) + es * i, es);
    ld_put(static_cast<uint8_t *>(out), i, x80_from_bits(b, dt));
  }
  return 0;
}

// numpy astype(longdouble -> dt)
int x80h_to(int dt, const void *a, void *dst, size_t n) {
  const int es = dt_size(dt);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t b = x80_to_bits(ld_at(static_cast<const uint8_t *>(a), i), dt);
    memcpy(static_cast<uint8_t *>(dst) + es * i, &b, es);
  }
  return 0;
}

// numpy's calendar datetime64 cast of n int64 ticks
int calh_convert(const int64_t *src, int64_t *dst, size_t n, int su, int64_t sn, int du, int64_t dn) {
  for (size_t i = 0; i < n; ++i) dst[i] = mc_cal_convert(src[i], su, sn, du, dn);
  return 0;
}

}  // extern "C"
