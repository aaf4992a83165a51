// mc_shuffle.hip -- Shuffle (byte transpose) encode/decode for gfx950.
//
// Reference: src/numcodecs/_shuffle.pyx:11-18 (_doShuffle) and :23-30
// (_doUnshuffle), driven by shuffle.py:40-58.  With count = nbytes / es:
//   encode: dst[b*count + i] = src[i*es + b]
//   decode: dst[i*es + b]    = src[b*count + i]
//
// Design (HBM-bound byte work, no MFMA):
//   * A tile is TE consecutive elements (TE = 4096 for es <= 8, 2048 for
//     es = 16): es*TE bytes on the element side, es planes of TE bytes on the
//     plane side.  One 256-thread workgroup moves one tile per iteration of a
//     grid-stride loop; each thread owns Q "quads" of 4 consecutive elements.
//   * A quad's es dwords are turned into its es plane dwords by a 4x4 byte
//     transpose in registers (v_perm_b32, mc_tr4), so every lane always moves
//     whole dwords.
//   * The element side is read/written with 16-B (es = 4, 8, 16) or 8-B
//     (es = 2) accesses per lane; the plane side either directly with one
//     dword per lane per plane (256 contiguous bytes per wave instruction) or
//     staged through LDS so that it too moves 16 B per lane (1 KiB per wave
//     instruction).  Which combination is fastest is measured
//     (tools/probe_enc.py, tools/probe_shuffle_tiles.py: interleaved
//     sweeps through the lab library) and the winner per (es, direction)
//     is the default.
//   * Sizes that are not a whole number of tiles finish with a generic
//     byte-granular kernel over the tail elements; unaligned buffers or
//     count % 4 != 0 run entirely on the generic kernel.
#include "mc_shuffle.h"

namespace {

// ---------------------------------------------------------------------------
// encode tile kernel
// ---------------------------------------------------------------------------
template <int ES, bool BITROUND, bool IN_LDS, bool OUT_LDS, bool NT, int QMUL = 1>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_enc(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    size_t ntiles, McBitRound br) {
  using G = Geom<ES, QMUL>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;

  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TE;

    uint32_t p[G::Q][ES];
    if constexpr (IN_LDS) {
      mc_u32x4 v[G::NV];
#pragma unroll
      for (int r = 0; r < G::NV; ++r)
        v[r] = mc_ld16<NT>(s + (size_t)(r * MC_BLOCK + tid) * 16);
#pragma unroll
      for (int r = 0; r < G::NV; ++r)
        reinterpret_cast<mc_u32x4 *>(lds)[r * MC_BLOCK + tid] = v[r];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < G::Q; ++q) {
        uint32_t w[ES];
        load_quad<ES, false>(lds + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w);
        if constexpr (BITROUND) mc_bitround_quad<ES>(w, br);
        mc_quad_to_planes<ES>(w, p[q]);
      }
      __syncthreads();
    } else {
      uint32_t w[G::Q][ES];
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
        load_quad<ES, NT>(s + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w[q]);
#pragma unroll
      for (int q = 0; q < G::Q; ++q) {
        if constexpr (BITROUND) mc_bitround_quad<ES>(w[q], br);
        mc_quad_to_planes<ES>(w[q], p[q]);
      }
    }

    if constexpr (OUT_LDS) {
      // plane-major image: plane b, quad qi -> dword b*(TE/4) + qi
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
#pragma unroll
        for (int b = 0; b < ES; ++b)
          reinterpret_cast<uint32_t *>(lds)[b * (G::TE / 4) + q * MC_BLOCK + tid] = p[q][b];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < G::NV; ++r) {
        const int u = r * MC_BLOCK + tid;
        const int b = u / G::PU;
        const int j = u - b * G::PU;
        const mc_u32x4 v = reinterpret_cast<const mc_u32x4 *>(lds)[u];
        mc_st16<NT>(d + (size_t)b * m.count + (size_t)j * 16, v);
      }
      __syncthreads();
    } else {
#pragma unroll
      for (int b = 0; b < ES; ++b)
#pragma unroll
        for (int q = 0; q < G::Q; ++q)
          mc_st4<NT>(d + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
    }
  }
}

// ---------------------------------------------------------------------------
// BitRound + Shuffle(4), the mask applied to the PLANES (C3, VERDICT r5 item
// 3).  BitRound's `& mask` is bytewise, so after the 4x4 byte transpose plane
// b only needs the mask's byte b: with Z = maskbits / 8 the planes below Z
// are zero (no transpose work) and only plane Z takes an `and` (maskbits %
// 8 != 0), against four `and`s and the full transpose per quad in
// k_shuffle_enc<4, true>: 16 instead of 20 VALU per quad at keepbits 10.
// Same tiles, loads and stores as k_shuffle_enc<4, BITROUND, false, false>.
// ---------------------------------------------------------------------------
template <int Z>
MC_DEV void mc_bitround_quad_planes4(const uint32_t (&w)[4], uint32_t (&p)[4], const McBitRound &br,
                                     uint32_t pmask) {
  uint32_t t[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = w[j] + ((w[j] >> br.maskbits) & 1u) + (uint32_t)br.half;
  const uint32_t a1 = mc_perm(t[1], t[0], 0x07030602u), a3 = mc_perm(t[3], t[2], 0x07030602u);
  if constexpr (Z < 2) {
    const uint32_t a0 = mc_perm(t[1], t[0], 0x05010400u), a2 = mc_perm(t[3], t[2], 0x05010400u);
    p[0] = Z == 0 ? (mc_perm(a2, a0, 0x05040100u) & pmask) : 0u;
    p[1] = Z == 1 ? (mc_perm(a2, a0, 0x07060302u) & pmask) : mc_perm(a2, a0, 0x07060302u);
  } else {
    p[0] = 0u;
    p[1] = 0u;
  }
  p[2] = Z == 2 ? (mc_perm(a3, a1, 0x05040100u) & pmask) : mc_perm(a3, a1, 0x05040100u);
  p[3] = mc_perm(a3, a1, 0x07060302u);
}

template <int Z, bool NT, int QMUL>
__global__ __launch_bounds__(MC_BLOCK) void k_bitround_shuffle4_planes(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles, McBitRound br,
    uint32_t pmask) {
  using G = Geom<4, QMUL>;
  const int tid = threadIdx.x;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TE;
    uint32_t w[G::Q][4], p[G::Q][4];
#pragma unroll
    for (int q = 0; q < G::Q; ++q) load_quad<4, NT>(s + (size_t)(q * MC_BLOCK + tid) * 16, w[q]);
#pragma unroll
    for (int q = 0; q < G::Q; ++q) mc_bitround_quad_planes4<Z>(w[q], p[q], br, pmask);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
        mc_st4<NT>(d + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4, p[q][b]);
  }
}

// ---------------------------------------------------------------------------
// decode tile kernel
// ---------------------------------------------------------------------------
template <int ES, bool IN_LDS, bool OUT_LDS, bool NT, int QMUL = 1>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_dec(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    size_t ntiles) {
  using G = Geom<ES, QMUL>;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x;

  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TE;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TB;

    uint32_t w[G::Q][ES];
    if constexpr (IN_LDS) {
      mc_u32x4 v[G::NV];
#pragma unroll
      for (int r = 0; r < G::NV; ++r) {
        const int u = r * MC_BLOCK + tid;
        const int b = u / G::PU;
        const int j = u - b * G::PU;
        v[r] = mc_ld16<NT>(s + (size_t)b * m.count + (size_t)j * 16);
      }
#pragma unroll
      for (int r = 0; r < G::NV; ++r)
        reinterpret_cast<mc_u32x4 *>(lds)[r * MC_BLOCK + tid] = v[r];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < G::Q; ++q) {
        uint32_t p[ES];
#pragma unroll
        for (int b = 0; b < ES; ++b)
          p[b] = reinterpret_cast<const uint32_t *>(lds)[b * (G::TE / 4) + q * MC_BLOCK + tid];
        mc_planes_to_quad<ES>(p, w[q]);
      }
      __syncthreads();
    } else {
      uint32_t p[G::Q][ES];
#pragma unroll
      for (int b = 0; b < ES; ++b)
#pragma unroll
        for (int q = 0; q < G::Q; ++q)
          p[q][b] = mc_ld4<NT>(s + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4);
#pragma unroll
      for (int q = 0; q < G::Q; ++q) mc_planes_to_quad<ES>(p[q], w[q]);
    }

    if constexpr (OUT_LDS) {
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
        store_quad<ES, false>(lds + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w[q]);
      __syncthreads();
#pragma unroll
      for (int r = 0; r < G::NV; ++r)
        mc_st16<NT>(d + (size_t)(r * MC_BLOCK + tid) * 16,
                    reinterpret_cast<const mc_u32x4 *>(lds)[r * MC_BLOCK + tid]);
      __syncthreads();
    } else {
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
        store_quad<ES, NT>(d + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w[q]);
    }
  }
}

// ---------------------------------------------------------------------------
// es = 8 with lane pairs: every lane moves 16 B per access on the element side
// (2 elements, lane-contiguous: 1 KiB per wave instruction).  Lanes 2m and
// 2m+1 hold elements 4m..4m+1 and 4m+2..4m+3; one pair-swap exchange
// gives the even lane the low dwords and the odd lane the high dwords of the
// 4 elements, and a 4x4 byte transpose turns them into plane dwords 0-3 (even)
// and 4-7 (odd).  A plane store instruction therefore writes two 128-B runs.
// Tile = 256 lanes x NV 16-B units.
// ---------------------------------------------------------------------------
// value of the partner lane (lane ^ 1): one DPP quad_perm [1,0,3,2] move
// (__shfl_xor(v, 1) compiles to an LDS ds_bpermute round trip)
MC_DEV uint32_t mc_pair_swap(uint32_t v) {  // value of the partner lane (lane ^ 1)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

template <bool BITROUND, bool NT, int NV>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle8_enc_pair(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles,
    McBitRound br) {
  constexpr int TB = NV * 16 * MC_BLOCK, TE = TB / 8;
  const int tid = threadIdx.x;
  const bool odd = tid & 1;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)TE;
    mc_u32x4 v[NV];
#pragma unroll
    for (int r = 0; r < NV; ++r) v[r] = mc_ld16<NT>(s + ((size_t)r * MC_BLOCK + tid) * 16);
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      mc_u32x4 x = v[r];
      if constexpr (BITROUND) {
        uint64_t e0 = mc_bitround64(((uint64_t)x.y << 32) | x.x, br);
        uint64_t e1 = mc_bitround64(((uint64_t)x.w << 32) | x.z, br);
        x = mc_u32x4{(uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1, (uint32_t)(e1 >> 32)};
      }
      const uint32_t a = mc_pair_swap(odd ? x.x : x.y);
      const uint32_t b = mc_pair_swap(odd ? x.z : x.w);
      uint32_t p0, p1, p2, p3;
      if (odd) mc_tr4(a, b, x.y, x.w, p0, p1, p2, p3);   // high dwords of e0..e3
      else mc_tr4(x.x, x.z, a, b, p0, p1, p2, p3);       // low dwords of e0..e3
      const size_t e = (size_t)r * (16 * MC_BLOCK / 8) + 4 * (size_t)(tid >> 1);
      uint8_t *pd = d + (odd ? 4 * m.count : 0) + e;
      mc_st4<NT>(pd, p0);
      mc_st4<NT>(pd + m.count, p1);
      mc_st4<NT>(pd + 2 * m.count, p2);
      mc_st4<NT>(pd + 3 * m.count, p3);
    }
  }
}

// es = 8, lane pairs + an LDS-staged plane side (round 5, layout V_PAIR_LDS):
// the pair layout's plane dwords (even lanes planes 0-3, odd lanes planes 4-7
// of 4 elements) go to a plane-major LDS image, and every lane then stores
// 16 B of one plane -- 1 KiB contiguous per wave store instruction, against
// two 128-B runs per instruction in the register layout.  Plane rows are
// padded to TE/4 + 8 dwords: a write instruction's even and odd lanes (planes
// b and b + 4, same quad index) then sit 32 banks apart, conflict-free, and
// rows stay 16-B aligned for the ds_read_b128s.
// Measured (tools/probe_enc_variants.py, 256 MiB): 99.7 us against 91.5 us
// for V_PAIR (BIG 108, BIG4 105, NO_NT 99.6): the LDS round trip costs more
// than the wider stores save.  Kept as a selectable variant, never the default.
template <bool BITROUND, bool NT, int NV>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle8_enc_pair_lds(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles,
    McBitRound br) {
  constexpr int TB = NV * 16 * MC_BLOCK, TE = TB / 8;
  constexpr int ROW = TE / 4 + 8;   // dwords per plane row in LDS
  constexpr int PU = TE / 16;       // 16-B units per plane
  __shared__ __attribute__((aligned(16))) uint32_t lds[8 * ROW];
  const int tid = threadIdx.x;
  const bool odd = tid & 1;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)TE;
    mc_u32x4 v[NV];
#pragma unroll
    for (int r = 0; r < NV; ++r) v[r] = mc_ld16<NT>(s + ((size_t)r * MC_BLOCK + tid) * 16);
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      mc_u32x4 x = v[r];
      if constexpr (BITROUND) {
        uint64_t e0 = mc_bitround64(((uint64_t)x.y << 32) | x.x, br);
        uint64_t e1 = mc_bitround64(((uint64_t)x.w << 32) | x.z, br);
        x = mc_u32x4{(uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1, (uint32_t)(e1 >> 32)};
      }
      const uint32_t a = mc_pair_swap(odd ? x.x : x.y);
      const uint32_t b = mc_pair_swap(odd ? x.z : x.w);
      uint32_t p0, p1, p2, p3;
      if (odd) mc_tr4(a, b, x.y, x.w, p0, p1, p2, p3);   // high dwords of e0..e3
      else mc_tr4(x.x, x.z, a, b, p0, p1, p2, p3);       // low dwords of e0..e3
      const int qi = r * (MC_BLOCK / 2) + (tid >> 1);    // quad index in the tile
      uint32_t *row = lds + (odd ? 4 * ROW : 0) + qi;
      row[0] = p0;
      row[ROW] = p1;
      row[2 * ROW] = p2;
      row[3 * ROW] = p3;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      const int u = r * MC_BLOCK + tid;
      const int pb = u / PU, j = u - pb * PU;
      const mc_u32x4 o = *reinterpret_cast<const mc_u32x4 *>(lds + pb * ROW + 4 * j);
      mc_st16<NT>(d + (size_t)pb * m.count + (size_t)j * 16, o);
    }
    __syncthreads();
  }
}

template <bool NT, int NV>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle8_dec_pair(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles) {
  constexpr int TB = NV * 16 * MC_BLOCK, TE = TB / 8;
  const int tid = threadIdx.x;
  const bool odd = tid & 1;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)TE;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)TB;
    uint32_t pl[NV][4];
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      const size_t e = (size_t)r * (16 * MC_BLOCK / 8) + 4 * (size_t)(tid >> 1);
      const uint8_t *ps = s + (odd ? 4 * m.count : 0) + e;
#pragma unroll
      for (int k = 0; k < 4; ++k) pl[r][k] = mc_ld4<NT>(ps + k * m.count);
    }
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      uint32_t w0, w1, w2, w3;  // even: low dwords of e0..e3; odd: high dwords
      mc_tr4(pl[r][0], pl[r][1], pl[r][2], pl[r][3], w0, w1, w2, w3);
      const uint32_t a = mc_pair_swap(odd ? w0 : w2);
      const uint32_t b = mc_pair_swap(odd ? w1 : w3);
      const mc_u32x4 o = odd ? mc_u32x4{a, w2, b, w3} : mc_u32x4{w0, a, w1, b};
      mc_st16<NT>(d + ((size_t)r * MC_BLOCK + tid) * 16, o);
    }
  }
}

// ---------------------------------------------------------------------------
// es = 8 with lane quads (V_WIDE, lab): lanes 4m..4m+3 hold elements
// 8m..8m+7 (2 each, 16 B, lane-contiguous as in the pair layout) and lane j
// of the quad owns planes j and j+4 of all 8 elements, so each plane access
// is 8 B per lane instead of the pair layout's 4 B.  The exchange is a 4x4
// all-to-all of dwords inside the quad: a byte transpose builds, per
// destination lane, the dword of that lane's plane bytes, then two DPP
// butterflies (quad_perm xor 1, xor 2; no LDS) deliver them.
// ---------------------------------------------------------------------------
template <int CTRL>
MC_DEV uint32_t mc_quad_dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// a[k] is destined to quad lane k; on return q[s] is what quad lane s sent here
MC_DEV void mc_quad_a2a(const uint32_t (&a)[4], uint32_t (&q)[4], int j) {
  const bool b0 = j & 1, b1 = j & 2;
  // xor 1: keep the items for lanes with my bit 0, trade the others
  const uint32_t r0 = mc_quad_dpp<0xB1>(b0 ? a[0] : a[1]);
  const uint32_t r1 = mc_quad_dpp<0xB1>(b0 ? a[2] : a[3]);
  // (from the even, from the odd lane of my pair) for destinations j&1 and (j&1)+2
  const uint32_t e_lo = b0 ? r0 : a[0], o_lo = b0 ? a[1] : r0;
  const uint32_t e_hi = b0 ? r1 : a[2], o_hi = b0 ? a[3] : r1;
  // xor 2: keep the destination with my bit 1, trade the other
  const uint32_t u0 = mc_quad_dpp<0x4E>(b1 ? e_lo : e_hi);
  const uint32_t u1 = mc_quad_dpp<0x4E>(b1 ? o_lo : o_hi);
  q[0] = b1 ? u0 : e_lo;
  q[1] = b1 ? u1 : o_lo;
  q[2] = b1 ? e_hi : u0;
  q[3] = b1 ? o_hi : u1;
}

template <bool BITROUND, bool NT, int NV>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle8_enc_quad(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles,
    McBitRound br) {
  constexpr int TB = NV * 16 * MC_BLOCK, TE = TB / 8;
  const int tid = threadIdx.x, j = tid & 3;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)TE;
    mc_u32x4 v[NV];
#pragma unroll
    for (int r = 0; r < NV; ++r) v[r] = mc_ld16<NT>(s + ((size_t)r * MC_BLOCK + tid) * 16);
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      mc_u32x4 x = v[r];
      if constexpr (BITROUND) {
        uint64_t e0 = mc_bitround64(((uint64_t)x.y << 32) | x.x, br);
        uint64_t e1 = mc_bitround64(((uint64_t)x.w << 32) | x.z, br);
        x = mc_u32x4{(uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1, (uint32_t)(e1 >> 32)};
      }
      // a[k] = byte k of (lo e0, lo e1, hi e0, hi e1): quad lane k's planes k, k+4
      uint32_t a[4], q[4];
      mc_tr4(x.x, x.z, x.y, x.w, a[0], a[1], a[2], a[3]);
      mc_quad_a2a(a, q, j);
      // q[s] = (plane j of elements 2s, 2s+1 | plane j+4 of the same two)
      const uint32_t l0 = mc_perm(q[1], q[0], 0x05040100u), l1 = mc_perm(q[3], q[2], 0x05040100u);
      const uint32_t h0 = mc_perm(q[1], q[0], 0x07060302u), h1 = mc_perm(q[3], q[2], 0x07060302u);
      const size_t e = (size_t)r * (16 * MC_BLOCK / 8) + 8 * (size_t)(tid >> 2);
      uint8_t *pd = d + (size_t)j * m.count + e;
      mc_st8<NT>(pd, mc_u32x2{l0, l1});
      mc_st8<NT>(pd + 4 * m.count, mc_u32x2{h0, h1});
    }
  }
}

template <bool NT, int NV>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle8_dec_quad(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles) {
  constexpr int TB = NV * 16 * MC_BLOCK, TE = TB / 8;
  const int tid = threadIdx.x, j = tid & 3;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)TE;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)TB;
    mc_u32x2 lo[NV], hi[NV];
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      const size_t e = (size_t)r * (16 * MC_BLOCK / 8) + 8 * (size_t)(tid >> 2);
      const uint8_t *ps = s + (size_t)j * m.count + e;
      lo[r] = mc_ld8<NT>(ps);
      hi[r] = mc_ld8<NT>(ps + 4 * m.count);
    }
#pragma unroll
    for (int r = 0; r < NV; ++r) {
      // a[s] = (plane j | plane j+4 bytes of elements 2s, 2s+1): quad lane s's
      uint32_t a[4], q[4];
      a[0] = mc_perm(hi[r].x, lo[r].x, 0x05040100u);
      a[1] = mc_perm(hi[r].x, lo[r].x, 0x07060302u);
      a[2] = mc_perm(hi[r].y, lo[r].y, 0x05040100u);
      a[3] = mc_perm(hi[r].y, lo[r].y, 0x07060302u);
      mc_quad_a2a(a, q, j);
      // q[k] = byte k of (lo e0, lo e1, hi e0, hi e1) of my two elements
      uint32_t lo0, lo1, hi0, hi1;
      mc_tr4(q[0], q[1], q[2], q[3], lo0, lo1, hi0, hi1);
      mc_st16<NT>(d + ((size_t)r * MC_BLOCK + tid) * 16, mc_u32x4{lo0, hi0, lo1, hi1});
    }
  }
}

// ---------------------------------------------------------------------------
// es = 4 with lane pairs on the plane side: lanes 2j and 2j+1 hold the quads
// of 8 consecutive elements; one DPP pair swap (quad_perm [1,0,3,2], no LDS)
// of two plane dwords lets the even lane own planes 0-1 and the odd lane
// planes 2-3 of all 8 elements, so each plane access is 8 B per lane (one
// store/load instruction writes/reads two 256-B runs) and a quad needs 2
// plane instructions instead of 4.  Element side unchanged (16 B per lane,
// lane-contiguous).
// ---------------------------------------------------------------------------

template <bool BITROUND, bool NT, int QMUL>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle4_enc_pair(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles,
    McBitRound br) {
  using G = Geom<4, QMUL>;
  const int tid = threadIdx.x;
  const bool odd = tid & 1;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TE + (odd ? 2 * m.count : 0);
    uint32_t w[G::Q][4];
#pragma unroll
    for (int q = 0; q < G::Q; ++q) load_quad<4, NT>(s + (size_t)(q * MC_BLOCK + tid) * 16, w[q]);
#pragma unroll
    for (int q = 0; q < G::Q; ++q) {
      if constexpr (BITROUND) mc_bitround_quad<4>(w[q], br);
      uint32_t p[4];
      mc_quad_to_planes<4>(w[q], p);
      // even keeps planes 0,1 and receives the odd lane's; odd keeps 2,3
      const uint32_t r0 = mc_pair_swap(odd ? p[0] : p[2]);
      const uint32_t r1 = mc_pair_swap(odd ? p[1] : p[3]);
      const mc_u32x2 a = odd ? mc_u32x2{r0, p[2]} : mc_u32x2{p[0], r0};
      const mc_u32x2 b = odd ? mc_u32x2{r1, p[3]} : mc_u32x2{p[1], r1};
      uint8_t *pd = d + (size_t)(q * MC_BLOCK + (tid & ~1)) * 4;  // 8-B aligned pair base
      mc_st8<NT>(pd, a);
      mc_st8<NT>(pd + m.count, b);
    }
  }
}

// ---------------------------------------------------------------------------
// es = 4 with 16-B plane stores (V_WIDE, lab): a thread owns groups of 4
// consecutive quads (16 elements, 64 B), loaded as 4 16-B vectors at a 64-B
// lane stride (the 4 load instructions of a group cover 16 KiB of the wave's
// tile contiguously between them); the 4 quads' plane dwords of plane b are
// 16 consecutive plane bytes, so every plane store is 16 B per lane, 1 KiB
// contiguous per wave instruction.  Same tiles as k_shuffle_enc<4, QMUL>.
// ---------------------------------------------------------------------------
template <bool BITROUND, bool NT, int QMUL>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle4_enc_wide(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles,
    McBitRound br) {
  using G = Geom<4, QMUL>;
  static_assert(G::Q == 4 * QMUL, "4 quads per group");
  const int tid = threadIdx.x;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TB;
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TE;
    uint32_t w[QMUL][4][4];
#pragma unroll
    for (int g = 0; g < QMUL; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) load_quad<4, NT>(s + (size_t)(g * MC_BLOCK + tid) * 64 + 16 * j, w[g][j]);
#pragma unroll
    for (int g = 0; g < QMUL; ++g) {
      uint32_t pl[4][4];  // [plane][quad]
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (BITROUND) mc_bitround_quad<4>(w[g][j], br);
        uint32_t p[4];
        mc_quad_to_planes<4>(w[g][j], p);
#pragma unroll
        for (int b = 0; b < 4; ++b) pl[b][j] = p[b];
      }
#pragma unroll
      for (int b = 0; b < 4; ++b)
        mc_st16<NT>(d + (size_t)b * m.count + (size_t)(g * MC_BLOCK + tid) * 16,
                    mc_u32x4{pl[b][0], pl[b][1], pl[b][2], pl[b][3]});
    }
  }
}

template <bool NT, int QMUL>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle4_dec_pair(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m, size_t ntiles) {
  using G = Geom<4, QMUL>;
  const int tid = threadIdx.x;
  const bool odd = tid & 1;
  MC_FOR_TILES(tile, ntiles, m) {
    const size_t c = tile / m.tiles_per_chunk;
    const size_t t = tile - c * m.tiles_per_chunk;
    const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TE + (odd ? 2 * m.count : 0);
    uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TB;
    mc_u32x2 a[G::Q], b[G::Q];
#pragma unroll
    for (int q = 0; q < G::Q; ++q) {
      const uint8_t *ps = s + (size_t)(q * MC_BLOCK + (tid & ~1)) * 4;
      a[q] = mc_ld8<NT>(ps);
      b[q] = mc_ld8<NT>(ps + m.count);
    }
#pragma unroll
    for (int q = 0; q < G::Q; ++q) {
      // even holds planes 0,1 of both quads (.x = its own quad, .y = odd's);
      // odd holds planes 2,3
      const uint32_t r0 = mc_pair_swap(odd ? a[q].x : a[q].y);
      const uint32_t r1 = mc_pair_swap(odd ? b[q].x : b[q].y);
      uint32_t p[4], w[4];
      if (odd) { p[0] = r0; p[1] = r1; p[2] = a[q].y; p[3] = b[q].y; }
      else { p[0] = a[q].x; p[1] = b[q].x; p[2] = r0; p[3] = r1; }
      mc_planes_to_quad<4>(p, w);
      store_quad<4, NT>(d + (size_t)(q * MC_BLOCK + tid) * 16, w);
    }
  }
}

// ---------------------------------------------------------------------------
// software-pipelined persistent variants (register layout): the next tile's
// loads are issued before this tile's stores, so waiting for them does not
// wait for the stores (vmcnt retires loads and stores in issue order).
// ---------------------------------------------------------------------------
template <int ES, bool BITROUND, bool NT, int QMUL>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_enc_pipe(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    size_t ntiles, McBitRound br) {
  using G = Geom<ES, QMUL>;
  const int tid = threadIdx.x;
  size_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto src_of = [&](size_t tl) {
    const size_t c = tl / m.tiles_per_chunk;
    return src + c * m.src_stride + (tl - c * m.tiles_per_chunk) * (size_t)G::TB;
  };
  uint32_t w[G::Q][ES];
  {
    const uint8_t *s = src_of(tile);
#pragma unroll
    for (int q = 0; q < G::Q; ++q)
      load_quad<ES, NT>(s + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w[q]);
  }
  for (;;) {
    const size_t nxt = tile + gridDim.x;
    uint32_t wn[G::Q][ES];
    if (nxt < ntiles) {
      const uint8_t *s = src_of(nxt);
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
        load_quad<ES, NT>(s + (size_t)(q * MC_BLOCK + tid) * 4 * ES, wn[q]);
    }
    const size_t c = tile / m.tiles_per_chunk;
    uint8_t *d = dst + c * m.dst_stride + (tile - c * m.tiles_per_chunk) * (size_t)G::TE;
#pragma unroll
    for (int q = 0; q < G::Q; ++q) {
      uint32_t pl[ES];
      if constexpr (BITROUND) mc_bitround_quad<ES>(w[q], br);
      mc_quad_to_planes<ES>(w[q], pl);
#pragma unroll
      for (int b = 0; b < ES; ++b)
        mc_st4<NT>(d + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4, pl[b]);
    }
    if (nxt >= ntiles) break;
#pragma unroll
    for (int q = 0; q < G::Q; ++q)
#pragma unroll
      for (int k = 0; k < ES; ++k) w[q][k] = wn[q][k];
    tile = nxt;
  }
}

template <int ES, bool NT, int QMUL>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_dec_pipe(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    size_t ntiles) {
  using G = Geom<ES, QMUL>;
  const int tid = threadIdx.x;
  size_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto src_of = [&](size_t tl) {
    const size_t c = tl / m.tiles_per_chunk;
    return src + c * m.src_stride + (tl - c * m.tiles_per_chunk) * (size_t)G::TE;
  };
  uint32_t p[G::Q][ES];
  {
    const uint8_t *s = src_of(tile);
#pragma unroll
    for (int b = 0; b < ES; ++b)
#pragma unroll
      for (int q = 0; q < G::Q; ++q)
        p[q][b] = mc_ld4<NT>(s + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4);
  }
  for (;;) {
    const size_t nxt = tile + gridDim.x;
    uint32_t pn[G::Q][ES];
    if (nxt < ntiles) {
      const uint8_t *s = src_of(nxt);
#pragma unroll
      for (int b = 0; b < ES; ++b)
#pragma unroll
        for (int q = 0; q < G::Q; ++q)
          pn[q][b] = mc_ld4<NT>(s + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4);
    }
    const size_t c = tile / m.tiles_per_chunk;
    uint8_t *d = dst + c * m.dst_stride + (tile - c * m.tiles_per_chunk) * (size_t)G::TB;
#pragma unroll
    for (int q = 0; q < G::Q; ++q) {
      uint32_t w[ES];
      mc_planes_to_quad<ES>(p[q], w);
      store_quad<ES, NT>(d + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w);
    }
    if (nxt >= ntiles) break;
#pragma unroll
    for (int q = 0; q < G::Q; ++q)
#pragma unroll
      for (int k = 0; k < ES; ++k) p[q][k] = pn[q][k];
    tile = nxt;
  }
}

// ---------------------------------------------------------------------------
// generic byte-granular kernels (any es >= 2, any count, any alignment):
// elements [e_begin, count) of every chunk.
// ---------------------------------------------------------------------------
template <bool BITROUND>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_enc_generic(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    size_t es, size_t e_begin, size_t nchunks, McBitRound br) {
  const size_t span = m.count - e_begin;
  const size_t total = span * nchunks;
  for (size_t idx = (size_t)blockIdx.x * MC_BLOCK + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * MC_BLOCK) {
    const size_t c = idx / span;
    const size_t i = e_begin + (idx - c * span);
    const uint8_t *s = src + c * m.src_stride + i * es;
    uint8_t *d = dst + c * m.dst_stride + i;
    if constexpr (BITROUND) {
      uint64_t v = 0;
      for (size_t b = 0; b < es; ++b) v |= (uint64_t)s[b] << (8 * b);
      if (es == 2) v = mc_bitround16x2((uint32_t)v, br) & 0xffffu;
      else if (es == 4) v = mc_bitround32((uint32_t)v, br);
      else v = mc_bitround64(v, br);
      for (size_t b = 0; b < es; ++b) d[b * m.count] = (uint8_t)(v >> (8 * b));
    } else {
      for (size_t b = 0; b < es; ++b) d[b * m.count] = s[b];
    }
  }
}

__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_dec_generic(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    size_t es, size_t e_begin, size_t nchunks) {
  const size_t span = m.count - e_begin;
  const size_t total = span * nchunks;
  for (size_t idx = (size_t)blockIdx.x * MC_BLOCK + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * MC_BLOCK) {
    const size_t c = idx / span;
    const size_t i = e_begin + (idx - c * span);
    const uint8_t *s = src + c * m.src_stride + i;
    uint8_t *d = dst + c * m.dst_stride + i * es;
    for (size_t b = 0; b < es; ++b) d[b] = s[b * m.count];
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
enum Variant { V_DEFAULT = 0, V_REG = 1, V_PLANE_LDS = 2, V_BOTH_LDS = 3, V_GENERIC = 4, V_PAIR = 5, V_WIDE = 6,
               V_PAIR_LDS = 7 };
// variant | V_NO_NT selects default-policy (temporal) global accesses
static constexpr int V_NO_NT = 8;
// variant | V_BIG selects 2x larger tiles, | V_BIG4 4x (register layout only)
static constexpr int V_BIG = 16;
static constexpr int V_BIG4 = 128;
// bits 5-6: log2 of the tile group taken per block step (MC_FOR_TILES)
static constexpr int V_GROUP_SHIFT = 5;
static constexpr int V_GROUP_MASK = 3 << V_GROUP_SHIFT;
// variant | V_PIPE: software-pipelined persistent loop (register layout only)
static constexpr int V_PIPE = 256;
// variant | V_BIG8 selects 8x larger tiles (register and lane-pair layouts)
static constexpr int V_BIG8 = 512;
static constexpr int V_TILE_MASK = V_BIG | V_BIG4 | V_BIG8;

// Measured defaults (tools/probe_enc.py, tools/probe_shuffle_tiles.py on
// MI355X, interleaved rounds; the sweeps are summarised in DESIGN.md).  Large
// buffers: one big tile per workgroup and a grid covering every tile (a
// looping workgroup waits for its previous tile's stores before it can use
// the next tile's loads, because vmcnt retires loads and stores in issue
// order).  Small buffers: 4096-element tiles so that there are enough
// workgroups.  A tile multiplier is only used where it leaves (almost) no
// elements to the byte-granular tail kernel: `count` a multiple of the
// tile, or at least 64 tiles per chunk.
static int tile_flag(size_t count, size_t base_elems, int want) {
  for (int flag = want; flag; flag = flag == V_BIG8 ? V_BIG4 : flag == V_BIG4 ? V_BIG : 0) {
    const size_t m = flag == V_BIG8 ? 8 : flag == V_BIG4 ? 4 : 2;
    if (count % (base_elems * m) == 0 || count >= 64 * base_elems * m) return flag;
  }
  return 0;
}

static int default_variant(size_t es, bool enc, size_t total_bytes, size_t count, size_t nchunks,
                           unsigned *grid_cap) {
  *grid_cap = 0x7fffffffu;
  if (total_bytes < ((size_t)64 << 20)) return V_REG;
  switch (es) {
    case 2: return V_REG | tile_flag(count, 4096, V_BIG4);  // 6.34 / 6.22 TB/s
    // encode of one chunk: 32768-element tiles (128 KiB per workgroup, 32
    // 16-B loads in flight per thread): 87.4 against 88.9 us for 64 KiB
    // tiles, 256 MiB (round 4, profiles/r04/probe_shuffle_tiles.json); a
    // batch of chunks under 64 MiB: lane pairs on 2x tiles, 256 x 1 MiB
    // 98.3 -> 85.5 us, 64 x 4 MiB 93.2 -> 85.0 us (the 128 KiB tiles lose
    // 6-13 % there, profiles/r04/probe_batch_variants.json); decode: lane
    // pairs, 8-B plane loads (5.96 vs 5.81 TB/s interleaved,
    // profiles/r01/shuffle4_pair_ab.log; larger pair tiles measured slower)
    case 4:
      if (enc && nchunks > 1 && count * 4 < ((size_t)64 << 20)) return V_PAIR | tile_flag(count, 4096, V_BIG);
      return enc ? (V_REG | tile_flag(count, 4096, V_BIG8)) : (V_PAIR | tile_flag(count, 4096, V_BIG));
    case 8:  // lane pairs keep the 8-B element side lane-contiguous
      return enc ? V_PAIR : (V_PAIR | tile_flag(count, 2048, V_BIG));  // 5.89 / 6.11 TB/s
    default:
      if (enc) return V_REG | tile_flag(count, 2048, V_BIG);
      *grid_cap = MC_MAX_GRID;
      return V_BOTH_LDS;
  }
}

template <int ES, bool BR, bool NT>
static void launch_enc_nt(int layout, const uint8_t *s, uint8_t *d, const ChunkMap &m,
                          size_t ntiles, unsigned grid, const McBitRound &br, hipStream_t st) {
  using G = Geom<ES>;
  if constexpr (ES == 4) {
    if ((layout & 7) == V_WIDE) {
      if (layout & V_BIG4) k_shuffle4_enc_wide<BR, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG) k_shuffle4_enc_wide<BR, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else k_shuffle4_enc_wide<BR, NT, 1><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      return;
    }
    if ((layout & 7) == V_PAIR) {
      if (layout & V_BIG8) k_shuffle4_enc_pair<BR, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG4) k_shuffle4_enc_pair<BR, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG) k_shuffle4_enc_pair<BR, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else k_shuffle4_enc_pair<BR, NT, 1><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      return;
    }
  }
  if constexpr (ES == 8) {
    if ((layout & 7) == V_WIDE) {
      if (layout & V_BIG4) k_shuffle8_enc_quad<BR, NT, 16><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG) k_shuffle8_enc_quad<BR, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else k_shuffle8_enc_quad<BR, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      return;
    }
    if ((layout & 7) == V_PAIR_LDS) {
      if (layout & V_BIG4) k_shuffle8_enc_pair_lds<BR, NT, 16><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG) k_shuffle8_enc_pair_lds<BR, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else k_shuffle8_enc_pair_lds<BR, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      return;
    }
    if ((layout & 7) == V_PAIR) {
      if (layout & V_BIG8) k_shuffle8_enc_pair<BR, NT, 32><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG4) k_shuffle8_enc_pair<BR, NT, 16><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else if (layout & V_BIG) k_shuffle8_enc_pair<BR, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      else k_shuffle8_enc_pair<BR, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
      return;
    }
  }
  if constexpr (ES == 4 && BR) {
    if ((layout == (V_REG | V_BIG8) || layout == (V_REG | V_BIG4) || layout == (V_REG | V_BIG)) &&
        mc_sched.br_planes) {
      // C3: the mask applied per plane
      const int z = br.maskbits / 8;
      const uint32_t pmask = 0x01010101u * (uint32_t)((br.mask >> (8 * z)) & 0xffu);
      if (layout & V_BIG8) {
        if (z == 0) k_bitround_shuffle4_planes<0, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
        else if (z == 1) k_bitround_shuffle4_planes<1, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
        else k_bitround_shuffle4_planes<2, NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
      } else if (layout & V_BIG4) {
        if (z == 0) k_bitround_shuffle4_planes<0, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
        else if (z == 1) k_bitround_shuffle4_planes<1, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
        else k_bitround_shuffle4_planes<2, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
      } else {
        if (z == 0) k_bitround_shuffle4_planes<0, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
        else if (z == 1) k_bitround_shuffle4_planes<1, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
        else k_bitround_shuffle4_planes<2, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br, pmask);
      }
      return;
    }
  }
  if (layout == (V_REG | V_PIPE | V_BIG4))
    k_shuffle_enc_pipe<ES, BR, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == (V_REG | V_PIPE | V_BIG))
    k_shuffle_enc_pipe<ES, BR, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == (V_REG | V_PIPE))
    k_shuffle_enc_pipe<ES, BR, NT, 1><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == (V_REG | V_BIG8))
    k_shuffle_enc<ES, BR, false, false, NT, (ES <= 8 ? 8 : 4)><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == (V_REG | V_BIG4))
    k_shuffle_enc<ES, BR, false, false, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == (V_REG | V_BIG))
    k_shuffle_enc<ES, BR, false, false, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == V_REG)
    k_shuffle_enc<ES, BR, false, false, NT><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles, br);
  else if (layout == V_PLANE_LDS)
    k_shuffle_enc<ES, BR, false, true, NT><<<grid, MC_BLOCK, G::TB, st>>>(s, d, m, ntiles, br);
  else
    k_shuffle_enc<ES, BR, true, true, NT><<<grid, MC_BLOCK, G::TB, st>>>(s, d, m, ntiles, br);
}

template <int ES, bool BR>
static int launch_enc_tiles(int variant, const uint8_t *s, uint8_t *d, const ChunkMap &m,
                            size_t ntiles, unsigned grid, const McBitRound &br,
                            hipStream_t st) {
  const int layout = variant & (7 | V_TILE_MASK | V_PIPE);
  if ((layout & 7) < V_REG || (layout & 7) == V_GENERIC) return MC_EINVAL;
  if ((layout & 7) == V_PAIR && ES != 8 && ES != 4) return MC_EINVAL;
  if ((layout & 7) == V_PAIR_LDS && (ES != 8 || (layout & (V_PIPE | V_BIG8)))) return MC_EINVAL;
  if ((layout & 7) == V_WIDE && ((ES != 4 && ES != 8) || (layout & (V_PIPE | V_BIG8)))) return MC_EINVAL;
  if ((layout & V_BIG8) && (layout & V_PIPE)) return MC_EINVAL;
  if (variant & V_NO_NT) launch_enc_nt<ES, BR, false>(layout, s, d, m, ntiles, grid, br, st);
  else launch_enc_nt<ES, BR, true>(layout, s, d, m, ntiles, grid, br, st);
  return mc_last_launch();
}

template <int ES, bool NT>
static void launch_dec_nt(int layout, const uint8_t *s, uint8_t *d, const ChunkMap &m,
                          size_t ntiles, unsigned grid, hipStream_t st) {
  using G = Geom<ES>;
  if constexpr (ES == 4) {
    if ((layout & 7) == V_PAIR) {
      if (layout & V_BIG8) k_shuffle4_dec_pair<NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else if (layout & V_BIG4) k_shuffle4_dec_pair<NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else if (layout & V_BIG) k_shuffle4_dec_pair<NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else k_shuffle4_dec_pair<NT, 1><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      return;
    }
  }
  if constexpr (ES == 8) {
    if ((layout & 7) == V_WIDE) {
      if (layout & V_BIG4) k_shuffle8_dec_quad<NT, 16><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else if (layout & V_BIG) k_shuffle8_dec_quad<NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else k_shuffle8_dec_quad<NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      return;
    }
    if ((layout & 7) == V_PAIR) {
      if (layout & V_BIG8) k_shuffle8_dec_pair<NT, 32><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else if (layout & V_BIG4) k_shuffle8_dec_pair<NT, 16><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else if (layout & V_BIG) k_shuffle8_dec_pair<NT, 8><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      else k_shuffle8_dec_pair<NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
      return;
    }
  }
  if (layout == (V_REG | V_PIPE | V_BIG4))
    k_shuffle_dec_pipe<ES, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == (V_REG | V_PIPE | V_BIG))
    k_shuffle_dec_pipe<ES, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == (V_REG | V_PIPE))
    k_shuffle_dec_pipe<ES, NT, 1><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == (V_REG | V_BIG8))
    k_shuffle_dec<ES, false, false, NT, (ES <= 8 ? 8 : 4)><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == (V_REG | V_BIG4))
    k_shuffle_dec<ES, false, false, NT, 4><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == (V_REG | V_BIG))
    k_shuffle_dec<ES, false, false, NT, 2><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == V_REG)
    k_shuffle_dec<ES, false, false, NT><<<grid, MC_BLOCK, 0, st>>>(s, d, m, ntiles);
  else if (layout == V_PLANE_LDS)
    k_shuffle_dec<ES, true, false, NT><<<grid, MC_BLOCK, G::TB, st>>>(s, d, m, ntiles);
  else
    k_shuffle_dec<ES, true, true, NT><<<grid, MC_BLOCK, G::TB, st>>>(s, d, m, ntiles);
}

template <int ES>
static int launch_dec_tiles(int variant, const uint8_t *s, uint8_t *d, const ChunkMap &m,
                            size_t ntiles, unsigned grid, hipStream_t st) {
  const int layout = variant & (7 | V_TILE_MASK | V_PIPE);
  if ((layout & 7) < V_REG || (layout & 7) > V_WIDE || (layout & 7) == V_GENERIC) return MC_EINVAL;
  if ((layout & 7) == V_PAIR && ES != 8 && ES != 4) return MC_EINVAL;
  if ((layout & 7) == V_WIDE && (ES != 8 || (layout & (V_PIPE | V_BIG8)))) return MC_EINVAL;
  if ((layout & V_BIG8) && (layout & V_PIPE)) return MC_EINVAL;
  if (variant & V_NO_NT) launch_dec_nt<ES, false>(layout, s, d, m, ntiles, grid, st);
  else launch_dec_nt<ES, true>(layout, s, d, m, ntiles, grid, st);
  return mc_last_launch();
}

static size_t tile_elems(size_t es, int variant) {
  const size_t mul = (variant & V_BIG8) ? 8 : (variant & V_BIG4) ? 4 : (variant & V_BIG) ? 2 : 1;
  const bool pairish = (variant & 7) == V_PAIR || (variant & 7) == V_WIDE || (variant & 7) == V_PAIR_LDS;
  if (pairish && es == 4)  // Geom<4, QMUL> tiles
    return 4096 * mul;
  if (pairish)  // 256 lanes x NV 16-B units of 8-B elements
    return 2048 * mul;
  const size_t te = es >= 16 ? 2048 : 4096;
  if ((variant & 7) != V_REG) return te;
  return te * mul;
}

}  // namespace

// Shared driver for every shuffle entry point (also used by the fused ops).
int mc_shuffle_impl(const void *src_, size_t src_stride, void *dst_, size_t dst_stride,
                    size_t nchunks, size_t chunk_bytes, size_t es, bool enc,
                    int variant, int max_blocks, const McBitRound *br,
                    hipStream_t st) {
  if (nchunks == 0 || chunk_bytes == 0) return MC_OK;
  if (!src_ || !dst_) return MC_EINVAL;
  const uint8_t *src = static_cast<const uint8_t *>(src_);
  uint8_t *dst = static_cast<uint8_t *>(dst_);
  if (es == 0) es = 1;
  if (chunk_bytes % es != 0) return MC_EINVAL;
  if (nchunks > 1 && (src_stride < chunk_bytes || dst_stride < chunk_bytes)) return MC_EINVAL;

  if (es == 1 && br == nullptr) {  // "no shuffling needed" (shuffle.py:31-33)
    return mc_copy_rows_impl(src, src_stride, dst, dst_stride, chunk_bytes, nchunks, st);
  }

  ChunkMap m;
  m.count = chunk_bytes / es;
  m.src_stride = nchunks > 1 ? src_stride : 0;
  m.dst_stride = nchunks > 1 ? dst_stride : 0;
  m.group = 1;

  unsigned default_cap = MC_MAX_GRID;
  if (variant == V_DEFAULT) {
    variant = default_variant(es, enc, chunk_bytes * nchunks, m.count, nchunks, &default_cap);
    // BitRound + Shuffle(4) of a large chunk: the plane-masked kernel on 64
    // KiB tiles (half the registers of the 128 KiB tiles, twice the waves to
    // hide its BitRound VALU): 256 MiB 89.2-89.4 against 89.7-91.0 us for
    // 128 KiB tiles, 91.3-92.2 for the element-masked kernel, plain
    // Shuffle(4) 87.2-87.6 (profiles/r06/probe_c3_layouts*.json)
    if (br && es == 4 && variant == (V_REG | V_BIG8) && tile_flag(m.count, 4096, V_BIG4) == V_BIG4)
      variant = V_REG | V_BIG4;
    if (max_blocks <= 0) max_blocks = (int)default_cap;
  }
  const bool fast_es = es == 2 || es == 4 || es == 8 || es == 16;
  const bool aligned16 = ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0) &&
                         (m.src_stride % 16 == 0) && (m.dst_stride % 16 == 0);
  if (!fast_es || !aligned16 || m.count % 4 != 0 || (br && es == 16)) variant = V_GENERIC;
  // the 16-B plane-side accesses need 16-B aligned plane bases
  if ((variant & 7) != V_GENERIC && (variant & 7) != V_REG && (variant & 7) != V_PAIR &&
      m.count % 16 != 0)
    variant = V_REG | (variant & (V_NO_NT | V_TILE_MASK | V_GROUP_MASK | V_PIPE));

  size_t e_done = 0;
  McBitRound nobr{};
  const McBitRound &brr = br ? *br : nobr;
  if ((variant & 7) != V_GENERIC) {
    if ((variant & 7) == V_PAIR && es != 8 && es != 4) variant = V_REG | (variant & V_NO_NT);
    if ((variant & 7) == V_PAIR_LDS && (es != 8 || !enc)) variant = V_REG | (variant & V_NO_NT);
    if ((variant & 7) == V_WIDE && !(es == 8 || (es == 4 && enc))) variant = V_REG | (variant & V_NO_NT);
    if ((variant & 7) != V_REG && (variant & 7) != V_PAIR && (variant & 7) != V_WIDE && (variant & 7) != V_PAIR_LDS)
      variant &= ~(V_TILE_MASK | V_PIPE);
    if ((variant & 7) == V_PAIR || (variant & 7) == V_WIDE || (variant & 7) == V_PAIR_LDS) variant &= ~V_PIPE;
    if ((variant & 7) == V_WIDE || (variant & 7) == V_PAIR_LDS || es == 16) variant &= ~V_BIG8;
    if (variant & V_PIPE) variant &= ~(V_GROUP_MASK | V_BIG8);
    if (variant & V_BIG8) variant &= ~(V_BIG | V_BIG4);
    if (variant & V_BIG4) variant &= ~V_BIG;
    m.group = 1u << ((variant & V_GROUP_MASK) >> V_GROUP_SHIFT);
    const size_t te = tile_elems(es, variant);
    m.tiles_per_chunk = m.count / te;
    const size_t ntiles = m.tiles_per_chunk * nchunks;
    if (ntiles > 0) {
      unsigned cap = max_blocks > 0 ? (unsigned)max_blocks : MC_MAX_GRID;
      unsigned grid = mc_grid_for(ntiles, m.group, cap);
      int rc = MC_EINVAL;
      if (enc) {
        switch (es) {
          case 2: rc = br ? launch_enc_tiles<2, true>(variant, src, dst, m, ntiles, grid, brr, st)
                          : launch_enc_tiles<2, false>(variant, src, dst, m, ntiles, grid, brr, st); break;
          case 4: rc = br ? launch_enc_tiles<4, true>(variant, src, dst, m, ntiles, grid, brr, st)
                          : launch_enc_tiles<4, false>(variant, src, dst, m, ntiles, grid, brr, st); break;
          case 8: rc = br ? launch_enc_tiles<8, true>(variant, src, dst, m, ntiles, grid, brr, st)
                          : launch_enc_tiles<8, false>(variant, src, dst, m, ntiles, grid, brr, st); break;
          case 16: rc = launch_enc_tiles<16, false>(variant, src, dst, m, ntiles, grid, brr, st); break;
        }
      } else {
        switch (es) {
          case 2: rc = launch_dec_tiles<2>(variant, src, dst, m, ntiles, grid, st); break;
          case 4: rc = launch_dec_tiles<4>(variant, src, dst, m, ntiles, grid, st); break;
          case 8: rc = launch_dec_tiles<8>(variant, src, dst, m, ntiles, grid, st); break;
          case 16: rc = launch_dec_tiles<16>(variant, src, dst, m, ntiles, grid, st); break;
        }
      }
      if (rc != MC_OK) return rc;
    }
    e_done = m.tiles_per_chunk * te;
  }
  if (e_done < m.count) {
    m.tiles_per_chunk = 0;
    const size_t total = (m.count - e_done) * nchunks;
    const unsigned grid = mc_grid_for(total, MC_BLOCK);
    if (enc) {
      if (br) k_shuffle_enc_generic<true><<<grid, MC_BLOCK, 0, st>>>(src, dst, m, es, e_done, nchunks, brr);
      else k_shuffle_enc_generic<false><<<grid, MC_BLOCK, 0, st>>>(src, dst, m, es, e_done, nchunks, brr);
    } else {
      k_shuffle_dec_generic<<<grid, MC_BLOCK, 0, st>>>(src, dst, m, es, e_done, nchunks);
    }
    return mc_last_launch();
  }
  return MC_OK;
}

extern "C" {

int mc_shuffle(const void *src, void *dst, size_t nbytes, size_t elementsize,
               mc_stream_t stream) {
  return mc_shuffle_impl(src, 0, dst, 0, 1, nbytes, elementsize, true, V_DEFAULT, 0,
                         nullptr, (hipStream_t)stream);
}

int mc_unshuffle(const void *src, void *dst, size_t nbytes, size_t elementsize,
                 mc_stream_t stream) {
  return mc_shuffle_impl(src, 0, dst, 0, 1, nbytes, elementsize, false, V_DEFAULT, 0,
                         nullptr, (hipStream_t)stream);
}

int mc_shuffle_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                     size_t nchunks, size_t chunk_bytes, size_t elementsize,
                     mc_stream_t stream) {
  return mc_shuffle_impl(src, src_stride, dst, dst_stride, nchunks, chunk_bytes,
                         elementsize, true, V_DEFAULT, 0, nullptr, (hipStream_t)stream);
}

int mc_unshuffle_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                       size_t nchunks, size_t chunk_bytes, size_t elementsize,
                       mc_stream_t stream) {
  return mc_shuffle_impl(src, src_stride, dst, dst_stride, nchunks, chunk_bytes,
                         elementsize, false, V_DEFAULT, 0, nullptr, (hipStream_t)stream);
}

int mc_bitround_shuffle(const void *src, void *dst, size_t n, int itemsize, int keepbits,
                        mc_stream_t stream) {
  if (!(itemsize == 2 || itemsize == 4 || itemsize == 8)) return MC_EINVAL;
  const int mbits = itemsize == 2 ? 10 : itemsize == 4 ? 23 : 52;
  if (keepbits < 0 || keepbits > mbits) return MC_EINVAL;
  if (keepbits == mbits)  // identity rounding: plain shuffle
    return mc_shuffle(src, dst, n * (size_t)itemsize, (size_t)itemsize, stream);
  const McBitRound br = mc_make_bitround(itemsize, keepbits);
  return mc_shuffle_impl(src, 0, dst, 0, 1, n * (size_t)itemsize, (size_t)itemsize, true,
                         V_DEFAULT, 0, &br, (hipStream_t)stream);
}

}  // extern "C"
