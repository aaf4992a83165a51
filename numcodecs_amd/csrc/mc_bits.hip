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

// Aligned fast path: a workgroup packs 32 KiB of bools (8 steps of coalesced
// 16-B loads, 2 packed bytes per lane per step) into 4 KiB staged in LDS one
// byte later than their packed index, so that the header-shifted output
// (encoded byte 1 + j = packed byte j) leaves as aligned 16-B stores: lane t
// stores encoded bytes [P + 16t, P + 16t + 16) = packed [P + 16t - 1, ...).
// The byte before the block (packed P - 1, or the header for block 0) is
// recomputed by thread 0 from the 8 bools before the block.
constexpr int PB_STEPS = 8;
constexpr size_t PB_SRC = (size_t)PB_STEPS * MC_BLOCK * 16;  // 32 KiB of bools
constexpr size_t PB_OUT = PB_SRC / 8;                          // 4 KiB packed

__global__ __launch_bounds__(MC_BLOCK) void k_packbits_blk(const uint8_t *__restrict__ src,
                                                           uint8_t *__restrict__ dst, size_t n,
                                                           size_t out_bytes) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[PB_OUT + 8];
  const size_t B = (size_t)blockIdx.x * PB_SRC, P = (size_t)blockIdx.x * PB_OUT;
  const int t = threadIdx.x;
  mc_u32x4 v[PB_STEPS];
  if (B + PB_SRC <= n) {
    // a whole block in range: the loads unbranched, all in flight together
    // (bounds-branched, each was waited for before the next issued)
#pragma unroll
    for (int k = 0; k < PB_STEPS; ++k) v[k] = mc_ld16<true>(src + B + (size_t)k * MC_BLOCK * 16 + 16 * (size_t)t);
  } else {
#pragma unroll
    for (int k = 0; k < PB_STEPS; ++k) {
      const size_t pos = B + (size_t)k * MC_BLOCK * 16 + 16 * (size_t)t;
      if (pos + 16 <= n) {
        v[k] = mc_ld16<true>(src + pos);
      } else {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int j = 0; j < 16; ++j)
          if (pos + j < n) w[j >> 2] |= (uint32_t)src[pos + j] << (8 * (j & 3));
        v[k] = mc_u32x4{w[0], w[1], w[2], w[3]};
      }
    }
  }
#pragma unroll
  for (int k = 0; k < PB_STEPS; ++k) {
    const uint32_t lo = pack8(((uint64_t)v[k].y << 32) | v[k].x);
    const uint32_t hi = pack8(((uint64_t)v[k].w << 32) | v[k].z);
    *reinterpret_cast<uint16_t *>(lds + 4 + 2 * (k * MC_BLOCK + t)) = (uint16_t)(lo | (hi << 8));
  }
  if (t == 0)
    lds[3] = blockIdx.x == 0 ? (uint8_t)((8 - n % 8) % 8)
                             : (uint8_t)pack8(*reinterpret_cast<const uint64_t *>(src + B - 8));
  __syncthreads();
  const uint32_t *l32 = reinterpret_cast<const uint32_t *>(lds);
  uint32_t d[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) d[k] = l32[4 * t + k];
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], 3);
  const size_t o = P + 16 * (size_t)t;
  if (o + 16 <= out_bytes) {
    mc_st16<true>(dst + o, mc_u32x4{w[0], w[1], w[2], w[3]});
  } else {
    for (int q = 0; q < 16 && o + q < out_bytes; ++q) dst[o + q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
  }
  // the block's last packed byte belongs to encoded byte P + 4096, which the
  // next block writes; the last block writes it itself
  if (t == 0 && blockIdx.x + 1 == gridDim.x && P + PB_OUT < out_bytes) dst[P + PB_OUT] = lds[PB_OUT + 3];
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

// Aligned fast path for decode: every store instruction of a wave writes
// 1 KiB contiguously (lane l writes bools [o, o + 16) with o = base + 1024v +
// 16l); the 2 packed bytes behind them (encoded offsets 1 + o/8 and 2 + o/8)
// come from one 8-byte load at the dword boundary below and v_alignbyte.
template <int V>
__global__ __launch_bounds__(MC_BLOCK) void k_unpackbits_wide(const uint8_t *__restrict__ src,
                                                              size_t src_bytes,
                                                              uint8_t *__restrict__ dst, size_t n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t base = ((size_t)blockIdx.x * (MC_BLOCK / 64) + wave) * (1024 * V);
  uint32_t x[V];
  const size_t last_e = 1 + (base + 1024 * (size_t)V) / 8;  // past the wave's last packed byte pair
  if (base + 1024 * (size_t)V <= n && (last_e & ~(size_t)3) + 8 <= src_bytes) {
    // the wave's whole range in bounds: the loads unbranched, all in flight
    // together (bounds-branched, each was waited for before the next issued)
    mc_u32x2 w[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const size_t e = 1 + (base + 1024 * (size_t)v + 16 * (size_t)lane) / 8;
      __builtin_memcpy(&w[v], __builtin_assume_aligned(src + (e & ~(size_t)3), 4), 8);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const size_t e = 1 + (base + 1024 * (size_t)v + 16 * (size_t)lane) / 8;
      x[v] = __builtin_amdgcn_alignbyte(w[v].y, w[v].x, (uint32_t)(e & 3));
    }
  } else {
#pragma unroll
  for (int v = 0; v < V; ++v) {  // every load first
    const size_t o = base + 1024 * (size_t)v + 16 * (size_t)lane;
    const size_t e = 1 + o / 8;  // encoded offset of the first packed byte
    const size_t a = e & ~(size_t)3;
    if (o < n && a + 8 <= src_bytes) {
      mc_u32x2 w;  // dword aligned (a % 8 may be 4): dwordx2 at dword alignment
      __builtin_memcpy(&w, __builtin_assume_aligned(src + a, 4), 8);
      x[v] = __builtin_amdgcn_alignbyte(w.y, w.x, (uint32_t)(e - a));
    } else if (o < n) {
      x[v] = (uint32_t)src[e] | (e + 1 < src_bytes ? (uint32_t)src[e + 1] << 8 : 0u);
    } else {
      x[v] = 0;
    }
  }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const size_t o = base + 1024 * (size_t)v + 16 * (size_t)lane;
    const uint64_t lo = unpack8(x[v] & 0xffu), hi = unpack8((x[v] >> 8) & 0xffu);
    if (o + 16 <= n) {
      mc_st16<true>(dst + o, mc_u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)});
    } else if (o < n) {
      for (int i = 0; i < 16 && o + i < n; ++i) dst[o + i] = (uint8_t)((i < 8 ? lo : hi) >> (8 * (i & 7)));
    }
  }
}

}  // namespace

extern "C" {

int mc_packbits(const void *src, void *dst, size_t n, mc_stream_t stream) {
  if (!dst || (n && !src)) return MC_EINVAL;
  const size_t out_bytes = 1 + (n + 7) / 8;
  if (n > 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    const size_t blocks = (n + PB_SRC - 1) / PB_SRC;
    if (blocks > 0x7fffffffu) return MC_EINVAL;
    k_packbits_blk<<<(unsigned)blocks, MC_BLOCK, 0, (hipStream_t)stream>>>(
        static_cast<const uint8_t *>(src), static_cast<uint8_t *>(dst), n, out_bytes);
    return mc_last_launch();
  }
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
  // 4 KiB of bools per wave: 2, 8 and 16 KiB measured slower (65.7-71.0,
  // 71.2-71.9, 76.7-78.9 vs 66.6-66.8 us for 256 MiB); staging the packed
  // bytes through LDS with 16-B loads was slower too (78 us)
  constexpr int V = 4;
  if (((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 15) == 0) {
    const size_t per_block = (size_t)4 * 1024 * V;
    const size_t blocks = (n + per_block - 1) / per_block;
    if (blocks > 0x7fffffffu) return MC_EINVAL;
    k_unpackbits_wide<V><<<(unsigned)blocks, MC_BLOCK, 0, (hipStream_t)stream>>>(
        static_cast<const uint8_t *>(src), src_bytes, static_cast<uint8_t *>(dst), n);
    return mc_last_launch();
  }
  const size_t lanes = (n + 63) / 64;
  const size_t grid = (lanes + MC_BLOCK - 1) / MC_BLOCK;
  if (grid > 0x7fffffffu) return MC_EINVAL;
  k_unpackbits<<<(unsigned)grid, MC_BLOCK, 0, (hipStream_t)stream>>>(
      static_cast<const uint8_t *>(src), src_bytes, static_cast<uint8_t *>(dst), n,
      ((uintptr_t)src & 3) == 0, ((uintptr_t)dst & 15) == 0);
  return mc_last_launch();
}

}  // extern "C"
