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
 * Built with plain -O3 and no -march, like the reference's release build
 * (src/numcodecs/meson.build:245-254).
 */
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
