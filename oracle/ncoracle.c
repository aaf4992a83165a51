/*
 * ncoracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * native hot loops, used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as bench.py's cpu_baseline leg.  Never linked
 * into or called by the product (numcodecs_amd/).
 *
 * Restated from zarr-developers/numcodecs (src/numcodecs/):
 *   nco_shuffle      <- _shuffle.pyx:11-18  _doShuffle
 *   nco_unshuffle    <- _shuffle.pyx:23-30  _doUnshuffle
 *   nco_fletcher32   <- fletcher32.pyx:24-57 _fletcher32 (HDF5 H5checksum.c
 *                       algorithm: 360-word blocks, big-endian 16-bit words)
 *   nco_jenkins_lookup3 <- jenkins.pyx:93-325 (hashlittle as in HDF5)
 *   nco_crc32c       <- checksum32.py:189-209 CRC32C.checksum, which calls the
 *                       third-party google_crc32c / crc32c package (absent
 *                       here): CRC-32C (Castagnoli, reflected 0x82F63B78,
 *                       init/xorout 0xFFFFFFFF), restated bit by bit and pinned
 *                       by the reference's fixture/crc32c files.
 * Built with plain -O3 and no -march, like the reference's release build
 * (src/numcodecs/meson.build:245-254).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

void nco_shuffle(const uint8_t *src, uint8_t *des, size_t nbytes, size_t element_size) {
  const size_t count = nbytes / element_size;
  for (size_t i = 0; i < count; i++) {
    const size_t offset = i * element_size;
    for (size_t byte_index = 0; byte_index < element_size; byte_index++)
      des[byte_index * count + i] = src[offset + byte_index];
  }
}

void nco_unshuffle(const uint8_t *src, uint8_t *des, size_t nbytes, size_t element_size) {
  const size_t count = nbytes / element_size;
  for (size_t i = 0; i < element_size; i++) {
    const size_t offset = i * count;
    for (size_t byte_index = 0; byte_index < count; byte_index++)
      des[byte_index * element_size + i] = src[offset + byte_index];
  }
}

uint32_t nco_fletcher32(const uint8_t *data, size_t nbytes) {
  size_t len = nbytes / 2;
  uint32_t sum1 = 0, sum2 = 0;
  while (len) {
    size_t tlen = len > 360 ? 360 : len;
    len -= tlen;
    do {
      sum1 += (uint32_t)(((uint16_t)data[0]) << 8) | ((uint16_t)data[1]);
      data += 2;
      sum2 += sum1;
    } while (--tlen);
    sum1 = (sum1 & 0xffff) + (sum1 >> 16);
    sum2 = (sum2 & 0xffff) + (sum2 >> 16);
  }
  if (nbytes % 2) {
    sum1 += (uint32_t)(((uint16_t)data[0]) << 8);
    sum2 += sum1;
    sum1 = (sum1 & 0xffff) + (sum1 >> 16);
    sum2 = (sum2 & 0xffff) + (sum2 >> 16);
  }
  sum1 = (sum1 & 0xffff) + (sum1 >> 16);
  sum2 = (sum2 & 0xffff) + (sum2 >> 16);
  return (sum2 << 16) | sum1;
}

/* Batched twins used by the CPU baseline (one chunk stream per process). */
void nco_shuffle_batch(const uint8_t *src, uint8_t *des, size_t nchunks, size_t chunk_bytes,
                       size_t element_size) {
  for (size_t c = 0; c < nchunks; c++)
    nco_shuffle(src + c * chunk_bytes, des + c * chunk_bytes, chunk_bytes, element_size);
}

void nco_unshuffle_batch(const uint8_t *src, uint8_t *des, size_t nchunks, size_t chunk_bytes,
                         size_t element_size) {
  for (size_t c = 0; c < nchunks; c++)
    nco_unshuffle(src + c * chunk_bytes, des + c * chunk_bytes, chunk_bytes, element_size);
}

/* ---- numpy-semantics elementwise codecs (CPU baseline of C3/C4) ---------
 * The reference expresses these in numpy; restated here as scalar C loops
 * with numpy's numerics (checked bit-exact against tests/golden by
 * tests/test_oracle.py::test_c_restatement_*).  Each call is ONE pass, where
 * numpy makes several (BitRound: copy + 5 in-place ufunc passes; FSO: three
 * temporaries + cast), so these loops are a faster CPU than the reference's
 * own numpy path -- a conservative baseline. */

/* bitround.py:62-68 on the int32 view of float32 data:
 *   maskbits = 23 - keepbits; mask = -1 << maskbits (int32, wraps)
 *   b += ((b >> maskbits) & 1) + ((1 << (maskbits - 1)) - 1); b &= mask
 * numpy int32 arithmetic wraps: done in uint32.  0 <= keepbits < 23. */
void nco_bitround32(const uint32_t *src, uint32_t *dst, size_t n, int keepbits) {
  const unsigned maskbits = 23u - (unsigned)keepbits;
  const uint32_t mask = 0xFFFFFFFFu << maskbits;
  const uint32_t half = (1u << (maskbits - 1)) - 1u;
  for (size_t i = 0; i < n; i++) {
    uint32_t b = src[i];
    b += ((b >> maskbits) & 1u) + half;
    dst[i] = b & mask;
  }
}

/* numpy's float -> int32 cast on x86-64 (cvttss2si): NaN and out-of-range
 * values give INT32_MIN (the "integer indefinite"); int16 then truncates. */
static int32_t nco_cvtt_f32(float v) {
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
  return (int32_t)v;
}

/* fixedscaleoffset.py:91-97 with dtype '<f4', astype '<i2':
 *   enc = np.around((arr - offset) * scale).astype('<i2')
 * NEP 50: the Python scalars are weak, so both operations run in float32
 * with offset/scale rounded to float32 (the caller passes them so). */
void nco_fso_encode_f4_i2(const float *x, int16_t *out, size_t n, float offset, float scale) {
  for (size_t i = 0; i < n; i++) {
    const float v = rintf((x[i] - offset) * scale);
    out[i] = (int16_t)nco_cvtt_f32(v);
  }
}

/* fixedscaleoffset.py:107-110: dec = (enc / scale) + offset in float64
 * (int16 array / Python float promotes to float64), then astype('<f4'). */
void nco_fso_decode_i2_f4(const int16_t *enc, float *out, size_t n, double scale, double offset) {
  for (size_t i = 0; i < n; i++) out[i] = (float)(((double)enc[i] / scale) + offset);
}

/* delta.py:63-66 with dtype = astype = '<i2': enc[0] = x[0]; enc[1:] = np.diff(x)
 * (int16 subtraction wraps). */
void nco_delta_encode_i2(const int16_t *x, int16_t *out, size_t n) {
  if (n == 0) return;
  out[0] = x[0];
  for (size_t i = 1; i < n; i++) out[i] = (int16_t)(uint16_t)((uint16_t)x[i] - (uint16_t)x[i - 1]);
}

/* delta.py:80: np.cumsum(enc, out=dec) accumulated in int16 (wraps). */
void nco_delta_decode_i2(const int16_t *enc, int16_t *out, size_t n) {
  uint16_t run = 0;
  for (size_t i = 0; i < n; i++) {
    run = (uint16_t)(run + (uint16_t)enc[i]);
    out[i] = (int16_t)run;
  }
}

/* ---- jenkins.pyx:93-325 ------------------------------------------------ */
static uint32_t nco_rot(uint32_t x, int k) { return (x << k) ^ (x >> (32 - k)); }

uint32_t nco_jenkins_lookup3(const uint8_t *k, size_t length, uint32_t initval) {
  uint32_t a, b, c;
  a = b = c = 0xdeadbeefu + (uint32_t)length + initval;
  if (length == 0) return c;
  while (length > 12) {
    a += k[0] + ((uint32_t)k[1] << 8) + ((uint32_t)k[2] << 16) + ((uint32_t)k[3] << 24);
    b += k[4] + ((uint32_t)k[5] << 8) + ((uint32_t)k[6] << 16) + ((uint32_t)k[7] << 24);
    c += k[8] + ((uint32_t)k[9] << 8) + ((uint32_t)k[10] << 16) + ((uint32_t)k[11] << 24);
    a -= c; a ^= nco_rot(c, 4);  c += b;
    b -= a; b ^= nco_rot(a, 6);  a += c;
    c -= b; c ^= nco_rot(b, 8);  b += a;
    a -= c; a ^= nco_rot(c, 16); c += b;
    b -= a; b ^= nco_rot(a, 19); a += c;
    c -= b; c ^= nco_rot(b, 4);  b += a;
    length -= 12;
    k += 12;
  }
  /* last block: bytes 11..0 of a 1..12-byte tail (the fall-through chain) */
  for (size_t i = length; i-- > 0;) {
    const uint32_t v = (uint32_t)k[i] << (8 * (i & 3));
    if (i >= 8) c += v; else if (i >= 4) b += v; else a += v;
  }
  c ^= b; c -= nco_rot(b, 14);
  a ^= c; a -= nco_rot(c, 11);
  b ^= a; b -= nco_rot(a, 25);
  c ^= b; c -= nco_rot(b, 16);
  a ^= c; a -= nco_rot(c, 4);
  b ^= a; b -= nco_rot(a, 14);
  c ^= b; c -= nco_rot(b, 24);
  return c;
}

/* ---- CRC-32C, bit by bit ---------------------------------------------- */
uint32_t nco_crc32c(const uint8_t *p, size_t n, uint32_t value) {
  uint32_t c = ~value;
  for (size_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int j = 0; j < 8; j++) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
  }
  return ~c;
}
