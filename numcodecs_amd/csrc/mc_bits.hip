// mc_bits.hip -- PackBits (packbits.py:33-82): booleans <-> bits, MSB first,
// behind a 1-byte header holding the number of padding bits (np.packbits /
// np.unpackbits order: element 8j+k is bit 7-k of packed byte j).
//
// Both kernels are HBM-bound (9n/8 bytes moved).  Bit gathering uses two
// multiply tricks, checked exhaustively against numpy in tests:
//   pack:   h = per-byte "nonzero" flag in bit 7 of each byte of a u64 of 8
//           bools; ((h >> 7) * 0x8040201008040201) >> 56 puts byte k's flag at
//           bit 7-k (no two partial products overlap, so no carries);
//   unpack: ((p * 0x8040201008040201) & 0x8080808080808080) >> 7 spreads bit
//           7-k of p into byte k as 0/1.
#include "mc_common.h"

namespace {

constexpr uint64_t SPREAD = 0x8040201008040201ull;

MC_DEV uint32_t pack8(uint64_t x) {
  const uint64_t h = (((x & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | x) & 0x8080808080808080ull;
  return (uint32_t)(((h >> 7) * SPREAD) >> 56);
}
MC_DEV uint64_t unpack8(uint32_t p) { return ((p * SPREAD) & 0x8080808080808080ull) >> 7; }

MC_DEV uint64_t load8_masked(const uint8_t *s, size_t pos, size_t n, bool al8) {
  if (al8 && pos + 8 <= n) return *reinterpret_cast<const uint64_t *>(s + pos);
  uint64_t x = 0;
  for (int k = 0; k < 8; ++k)
    if (pos + k < n) x |= (uint64_t)s[pos + k] << (8 * k);
  return x;
}

// lane g writes encoded bytes [16g, 16g + 16): byte 0 = pad, byte 1 + j =
// pack(src[8j, 8j + 8)) with bools past n read as False.
__global__ __launch_bounds__(MC_BLOCK) void k_packbits(const uint8_t *__restrict__ src,
                                                       uint8_t *__restrict__ dst, size_t n,
                                                       size_t out_bytes, bool al8, bool dst_al16) {
  const size_t g = (size_t)blockIdx.x * MC_BLOCK + threadIdx.x;
  const size_t d0 = 16 * g;
  if (d0 >= out_bytes) return;
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const size_t j = d0 + q;
    uint32_t b;
    if (j == 0) b = (uint32_t)((8 - n % 8) % 8);
    else if (j < out_bytes) b = pack8(load8_masked(src, 8 * (j - 1), n, al8));
    else b = 0;
    w[q >> 2] |= b << (8 * (q & 3));
  }
  if (dst_al16 && d0 + 16 <= out_bytes) {
    mc_st16<false>(dst + d0, mc_u32x4{w[0], w[1], w[2], w[3]});
  } else {
    for (int q = 0; q < 16 && d0 + q < out_bytes; ++q) dst[d0 + q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
  }
}

// lane g writes bools [64g, 64g + 64) from packed bytes 8g..8g+7, which sit at
// encoded offsets 1 + 8g .. 8 + 8g (src = the encoded buffer, header first).
__global__ __launch_bounds__(MC_BLOCK) void k_unpackbits(const uint8_t *__restrict__ src,
                                                         size_t src_bytes, uint8_t *__restrict__ dst,
                                                         size_t n, bool src_al4, bool dst_al16) {
  const size_t g = (size_t)blockIdx.x * MC_BLOCK + threadIdx.x;
  const size_t o0 = 64 * g;
  if (o0 >= n) return;
  uint32_t lo, hi;
  if (src_al4 && 8 * g + 12 <= src_bytes) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(src + 8 * g);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    lo = __builtin_amdgcn_alignbyte(w1, w0, 1);
    hi = __builtin_amdgcn_alignbyte(w2, w1, 1);
  } else {
    uint64_t x = 0;
    for (int k = 0; k < 8; ++k)
      if (1 + 8 * g + k < src_bytes) x |= (uint64_t)src[1 + 8 * g + k] << (8 * k);
    lo = (uint32_t)x;
    hi = (uint32_t)(x >> 32);
  }
  uint64_t o[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = unpack8(((k < 4 ? lo : hi) >> (8 * (k & 3))) & 0xffu);
  if (dst_al16 && o0 + 64 <= n) {
#pragma unroll
    for (int v = 0; v < 4; ++v)
      mc_st16<false>(dst + o0 + 16 * v, mc_u32x4{(uint32_t)o[2 * v], (uint32_t)(o[2 * v] >> 32),
                                                 (uint32_t)o[2 * v + 1], (uint32_t)(o[2 * v + 1] >> 32)});
  } else {
    for (int i = 0; i < 64 && o0 + i < n; ++i) dst[o0 + i] = (uint8_t)(o[i >> 3] >> (8 * (i & 7)));
  }
}

}  // namespace

extern "C" {

int mc_packbits(const void *src, void *dst, size_t n, mc_stream_t stream) {
  if (!dst || (n && !src)) return MC_EINVAL;
  const size_t out_bytes = 1 + (n + 7) / 8;
  const size_t lanes = (out_bytes + 15) / 16;
  const size_t grid = (lanes + MC_BLOCK - 1) / MC_BLOCK;
  if (grid > 0x7fffffffu) return MC_EINVAL;
  k_packbits<<<(unsigned)grid, MC_BLOCK, 0, (hipStream_t)stream>>>(
      static_cast<const uint8_t *>(src), static_cast<uint8_t *>(dst), n, out_bytes,
      ((uintptr_t)src & 7) == 0, ((uintptr_t)dst & 15) == 0);
  return mc_last_launch();
}

int mc_unpackbits(const void *src, size_t src_bytes, void *dst, size_t n, mc_stream_t stream) {
  if (src_bytes < 1 || !src || (n && !dst)) return MC_EINVAL;
  if (n > 8 * (src_bytes - 1)) return MC_EINVAL;
  if (n == 0) return MC_OK;
  const size_t lanes = (n + 63) / 64;
  const size_t grid = (lanes + MC_BLOCK - 1) / MC_BLOCK;
  if (grid > 0x7fffffffu) return MC_EINVAL;
  k_unpackbits<<<(unsigned)grid, MC_BLOCK, 0, (hipStream_t)stream>>>(
      static_cast<const uint8_t *>(src), src_bytes, static_cast<uint8_t *>(dst), n,
      ((uintptr_t)src & 3) == 0, ((uintptr_t)dst & 15) == 0);
  return mc_last_launch();
}

}  // extern "C"
