// lab_shuffle4.hip -- LAB ONLY (libmcodec_lab.so): alternative Shuffle(4)
// encode schedules measured against the product's k_shuffle_enc<4, ..., 4>
// (tools/probe_enc4_lab.py; tests/test_gpu_sweep.py keeps every one of them
// byte-identical to the reference transpose, _shuffle.pyx:11-18).
//
// Every kernel moves one tile of Q quads x 256 threads (Q = 16: 64 KiB) per
// workgroup, element side 16 B per lane (lane-contiguous, nontemporal):
//   kind 0  register staging, planes stored dword by dword (the product's
//           layout: plane-major store order)
//   kind 1  as 0, quad-major store order (the 4 planes of one quad row
//           back to back)
//   kind 2  as 0 with an XCD-aware tile order: workgroup b (dispatched to
//           XCD b % 8) takes tile (b % 8) * ntiles/8 + b / 8, so each XCD
//           streams one contiguous eighth of the chunk
//   kind 3  element side by LDS-DMA (global_load_lds_dwordx4, nontemporal
//           (aux = NT), straight into a lane-linear LDS image; each wave reads
//           back only what it loaded, so no barrier), Q = 16
//   kind 4  as 3 with Q = 8 (32 KiB of LDS per workgroup: more resident)
//   kind 5  as 3 with the XCD-aware order
//   kind 6  16-B plane stores: lanes 4m..4m+3 trade plane dwords with two
//           DPP butterflies so lane j owns plane j of 16 consecutive elements
//   kind 7  the access pattern alone: kind 0's loads and stores with no byte
//           transpose (not a shuffle; a ceiling for the layout)
//   kind 8  register staging, Q = 32 (two tiles' loads in flight per thread)
//   kind 9  as 4 with default-policy LDS-DMA loads
//   kind 10 as 8 with the quad-major store order
//   kind 11 register staging, Q = 64 (four tiles' loads in flight)
//   kinds 12-15  kind 8 (Q = 32, the product's tile) with the tiles spread:
//           workgroup b takes tile (b % S) * ntiles/S + b / S, so the
//           workgroups in flight write S far-apart regions of every plane
//           instead of one (S = 2, 4, 16, 64)
//   kind 16  kind 8 with the plane store order rotated per workgroup
//           (workgroup b stores planes b, b+1, b+2, b+3 mod 4), so the
//           workgroups in flight spread their stores over all 4 planes
//   kind 17  as 16, quad-major order with the rotation
//   kind 18  kind 8 with default-policy (temporal) plane stores and
//           nontemporal loads: the Infinity Cache takes the 4 plane streams
//           and writes them back in its own order
//   kind 19  kind 8 with default-policy loads and nontemporal stores
#include "mc_shuffle.h"

#include <type_traits>

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

MC_DEV size_t lab_tile(int spread, size_t ntiles) {
  const size_t b = blockIdx.x;
  if (spread <= 1) return b;
  const size_t per = ntiles / spread;  // the host checks ntiles % spread == 0
  return (b % spread) * per + b / spread;
}

template <int Q, int ORDER, int XCD, bool PERM, bool LDNT = true, bool STNT = true>
__global__ __launch_bounds__(MC_BLOCK) void k_lab_enc4_reg(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                          size_t count, size_t ntiles) {
  constexpr size_t TE = (size_t)Q * 4 * MC_BLOCK;
  const int tid = threadIdx.x;
  const size_t tile = lab_tile(XCD, ntiles);
  const uint8_t *s = src + tile * TE * 4;
  uint8_t *d = dst + tile * TE;
  uint32_t w[Q][4], p[Q][4];
#pragma unroll
  for (int q = 0; q < Q; ++q) load_quad<4, LDNT>(s + (size_t)(q * MC_BLOCK + tid) * 16, w[q]);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    if constexpr (PERM) mc_quad_to_planes<4>(w[q], p[q]);
    else
#pragma unroll
      for (int b = 0; b < 4; ++b) p[q][b] = w[q][b];
  }
  if constexpr (ORDER == 2 || ORDER == 3) {
    auto rot = [&](auto R) {
      constexpr int r = decltype(R)::value;
      if constexpr (ORDER == 2) {
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            const int b = (bb + r) & 3;
            mc_st4<true>(d + (size_t)b * count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
          }
      } else {
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) {
            const int b = (bb + r) & 3;
            mc_st4<true>(d + (size_t)b * count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
          }
      }
    };
    switch (blockIdx.x & 3) {
      case 0: rot(std::integral_constant<int, 0>{}); break;
      case 1: rot(std::integral_constant<int, 1>{}); break;
      case 2: rot(std::integral_constant<int, 2>{}); break;
      default: rot(std::integral_constant<int, 3>{}); break;
    }
  } else if constexpr (ORDER == 0) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < Q; ++q) mc_st4<STNT>(d + (size_t)b * count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
  } else {
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b) mc_st4<true>(d + (size_t)b * count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
  }
}

template <int Q, int XCD, int AUX>
__global__ __launch_bounds__(MC_BLOCK) void k_lab_enc4_glds(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                           size_t count, size_t ntiles) {
  constexpr size_t TE = (size_t)Q * 4 * MC_BLOCK;
  __shared__ __attribute__((aligned(16))) uint8_t img[Q * MC_BLOCK * 16];
  const int tid = threadIdx.x, wave = tid >> 6;
  const size_t tile = lab_tile(XCD, ntiles);
  const uint8_t *s = src + tile * TE * 4;
  uint8_t *d = dst + tile * TE;
  // wave w's 16-B units of quad row q land at img + (q*256 + 64w)*16 + 16*lane
#pragma unroll
  for (int q = 0; q < Q; ++q)
    __builtin_amdgcn_global_load_lds((glb_void *)(s + (size_t)(q * MC_BLOCK + tid) * 16),
                                     (lds_void *)(img + (q * MC_BLOCK + wave * 64) * 16), 16, 0, AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t p[Q][4];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const mc_u32x4 v = *reinterpret_cast<const mc_u32x4 *>(img + (q * MC_BLOCK + tid) * 16);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    mc_quad_to_planes<4>(w, p[q]);
  }
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int q = 0; q < Q; ++q) mc_st4<true>(d + (size_t)b * count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
}

template <int CTRL>
MC_DEV uint32_t lab_quad_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// a[k] is destined to quad lane k; on return q[s] is what quad lane s sent here
MC_DEV void lab_quad_a2a(const uint32_t (&a)[4], uint32_t (&q)[4], int j) {
  const bool b0 = j & 1, b1 = j & 2;
  const uint32_t r0 = lab_quad_dpp<0xB1>(b0 ? a[0] : a[1]);
  const uint32_t r1 = lab_quad_dpp<0xB1>(b0 ? a[2] : a[3]);
  const uint32_t e_lo = b0 ? r0 : a[0], o_lo = b0 ? a[1] : r0;
  const uint32_t e_hi = b0 ? r1 : a[2], o_hi = b0 ? a[3] : r1;
  const uint32_t u0 = lab_quad_dpp<0x4E>(b1 ? e_lo : e_hi);
  const uint32_t u1 = lab_quad_dpp<0x4E>(b1 ? o_lo : o_hi);
  q[0] = b1 ? u0 : e_lo;
  q[1] = b1 ? u1 : o_lo;
  q[2] = b1 ? e_hi : u0;
  q[3] = b1 ? o_hi : u1;
}

template <int Q>
__global__ __launch_bounds__(MC_BLOCK) void k_lab_enc4_quadlane(const uint8_t *__restrict__ src,
                                                               uint8_t *__restrict__ dst, size_t count) {
  constexpr size_t TE = (size_t)Q * 4 * MC_BLOCK;
  const int tid = threadIdx.x, j = tid & 3;
  const uint8_t *s = src + (size_t)blockIdx.x * TE * 4;
  uint8_t *d = dst + (size_t)blockIdx.x * TE + (size_t)j * count;
  uint32_t w[Q][4];
#pragma unroll
  for (int q = 0; q < Q; ++q) load_quad<4, true>(s + (size_t)(q * MC_BLOCK + tid) * 16, w[q]);
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    uint32_t p[4], r[4];
    mc_quad_to_planes<4>(w[q], p);
    lab_quad_a2a(p, r, j);  // r[s] = plane j of quad lane s's 4 elements
    mc_st16<true>(d + (size_t)(q * MC_BLOCK + (tid & ~3)) * 4, mc_u32x4{r[0], r[1], r[2], r[3]});
  }
}

}  // namespace

extern "C" int mc_lab_shuffle4_enc(const void *src, void *dst, size_t nbytes, int kind, mc_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  const int Q = (kind == 4 || kind == 9) ? 8 : (kind == 8 || kind == 10 || kind >= 12) ? 32 : kind == 11 ? 64 : 16;
  const size_t tb = (size_t)Q * 4 * MC_BLOCK * 4;  // tile bytes
  if (!src || !dst || nbytes == 0 || nbytes % tb || (uintptr_t)src % 16 || (uintptr_t)dst % 16) return MC_EINVAL;
  const size_t count = nbytes / 4, ntiles = nbytes / tb;
  if ((kind == 2 || kind == 5) && ntiles % 8) return MC_EINVAL;
  if (kind >= 12 && kind <= 15 && ntiles % 64) return MC_EINVAL;
  const unsigned g = (unsigned)ntiles;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  switch (kind) {
    case 0: k_lab_enc4_reg<16, 0, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 1: k_lab_enc4_reg<16, 1, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 2: k_lab_enc4_reg<16, 0, 8, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 3: k_lab_enc4_glds<16, 0, 2><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 4: k_lab_enc4_glds<8, 0, 2><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 5: k_lab_enc4_glds<16, 8, 2><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 9: k_lab_enc4_glds<8, 0, 0><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 6: k_lab_enc4_quadlane<16><<<g, MC_BLOCK, 0, st>>>(s, d, count); break;
    case 7: k_lab_enc4_reg<16, 0, 0, false><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 8: k_lab_enc4_reg<32, 0, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 10: k_lab_enc4_reg<32, 1, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 11: k_lab_enc4_reg<64, 0, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 12: k_lab_enc4_reg<32, 0, 2, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 13: k_lab_enc4_reg<32, 0, 4, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 14: k_lab_enc4_reg<32, 0, 16, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 15: k_lab_enc4_reg<32, 0, 64, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 16: k_lab_enc4_reg<32, 2, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 17: k_lab_enc4_reg<32, 3, 0, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 18: k_lab_enc4_reg<32, 0, 0, true, true, false><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    case 19: k_lab_enc4_reg<32, 0, 0, true, false, true><<<g, MC_BLOCK, 0, st>>>(s, d, count, ntiles); break;
    default: return MC_EINVAL;
  }
  return mc_last_launch();
}
