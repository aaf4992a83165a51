// lab_crc.hip -- LAB ONLY (libmcodec_lab.so): the bit-sliced CRC tile kernel
// (mcck::k_crc_tiles_bs, checksum-only pass) with a deeper register ring and
// per-wave partials (tools/probe_crc_ring.py).  The product kernel folds one
// tile while the next is loaded (two register sets) and combines its four
// wave partials through LDS with one barrier per tile; its waves sat parked
// on waits 46 % of their cycles (SQ_WAIT_ANY, round 5).  Here:
//   R register sets: tiles i+1 .. i+R-1 in flight while tile i is folded;
//   WAVEP: each wave writes its own partial (parts[4 * tile + wave], XORed
//          by the caller), no LDS and no barrier; else the product's barrier.
// Single chunk, n a multiple of the tile size, 16-B aligned source.
#include "mc_checksum.h"

namespace mcck {
namespace {

template <int KIND, int K, int R, bool WAVEP>
__global__ __launch_bounds__(MC_BLOCK, 2) void k_lab_crc(const uint8_t *__restrict__ src, size_t total,
                                                         uint32_t *__restrict__ parts) {
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t gx[32];  // g * x^i, g = x^(-128 threadIdx.x)
  gx[0] = crc_consts<KIND>().g[threadIdx.x];
#pragma unroll
  for (int i = 1; i < 32; ++i) gx[i] = mulx_r<KIND>(gx[i - 1]);
  constexpr size_t TB = (size_t)K * STEP;
  mc_u32x4 v[R][K];
  auto load = [&](mc_u32x4 (&d)[K], size_t t) {
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = mc_ld16<true>(src + t * TB + 16 * (size_t)threadIdx.x + (size_t)k * STEP);
  };
  size_t tile = blockIdx.x;
  if (tile >= total) return;
#pragma unroll
  for (int r = 0; r + 1 < R; ++r)
    if (tile + (size_t)r * gridDim.x < total) load(v[r], tile + (size_t)r * gridDim.x);
  int par = 0;
  for (;;) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t tn = tile + (size_t)(R - 1) * gridDim.x;
      if (tn < total) load(v[(r + R - 1) % R], tn);
      const uint32_t acc = crc_fold_bs<KIND, K>(v[r]);
      uint32_t p = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i)
        p = __builtin_amdgcn_bitop3_b32(p, (uint32_t)__builtin_amdgcn_sbfe((int)acc, 31 - i, 1), gx[i], 0x78);
      p = wave_xor(p);
      if constexpr (WAVEP) {
        if (lane == 0) parts[4 * tile + wave] = p;
      } else {
        if (lane == 0) red[par][wave] = p;
        __syncthreads();
        if (threadIdx.x == 0) parts[tile] = red[par][0] ^ red[par][1] ^ red[par][2] ^ red[par][3];
        par ^= 1;
      }
      tile += gridDim.x;
      if (tile >= total) return;
    }
  }
}

template <int KIND>
int lab_crc_kind(const uint8_t *s, size_t total, int K, int R, bool wavep, unsigned grid, uint32_t *parts,
                 hipStream_t st) {
#define LC(KK, RR, WP) k_lab_crc<KIND, KK, RR, WP><<<grid, MC_BLOCK, 0, st>>>(s, total, parts)
  if (K == 16 && R == 2 && wavep) LC(16, 2, true);
  else if (K == 16 && R == 2) LC(16, 2, false);
  else if (K == 8 && R == 3 && wavep) LC(8, 3, true);
  else if (K == 8 && R == 3) LC(8, 3, false);
  else if (K == 8 && R == 4 && wavep) LC(8, 4, true);
  else if (K == 8 && R == 2 && wavep) LC(8, 2, true);
  else if (K == 16 && R == 3 && wavep) LC(16, 3, true);
  else return MC_EINVAL;
#undef LC
  return MC_OK;
}

}  // namespace
}  // namespace mcck

// kind MC_CK_CRC32 / MC_CK_CRC32C; n a multiple of K * 4096; wavep: parts
// holds 4 words per tile, else 1
extern "C" int mc_lab_crc(int kind, const void *src, size_t n, int K, int R, int wavep, unsigned grid,
                          uint32_t *parts, mc_stream_t stream) {
  const size_t tb = (size_t)K * mcck::STEP;
  if (!src || !parts || n == 0 || n % tb || ((uintptr_t)src & 15) || grid == 0) return MC_EINVAL;
  const size_t total = n / tb;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  hipStream_t st = (hipStream_t)stream;
  const int rc = kind == MC_CK_CRC32 ? mcck::lab_crc_kind<mcck::K_CRC32>(s, total, K, R, wavep != 0, grid, parts, st)
                 : kind == MC_CK_CRC32C ? mcck::lab_crc_kind<mcck::K_CRC32C>(s, total, K, R, wavep != 0, grid, parts, st)
                                        : MC_EINVAL;
  return rc != MC_OK ? rc : mc_last_launch();
}

// the product's checksum-only tile pass (tile partials, no finalize)
extern "C" int mc_lab_crc_product(int kind, const void *src, size_t n, int K, unsigned grid, uint32_t *parts,
                                  mc_stream_t stream) {
  const size_t tb = (size_t)K * mcck::STEP;
  if (!src || !parts || n == 0 || n % tb || grid == 0) return MC_EINVAL;
  const size_t total = n / tb;
  const mcck::CrcFin fin{};
  const int rc = mcck::launch_crc_bs(kind, K, 2, 2, static_cast<const uint8_t *>(src), 0, nullptr, 0, n, total,
                                     total, parts, fin, nullptr, grid, (hipStream_t)stream);
  return rc != MC_OK ? rc : mc_last_launch();
}
