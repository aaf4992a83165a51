// mc_shuffle.h -- tile geometry and quad I/O shared by the Shuffle kernels
// (mc_shuffle.hip) and the fused Shuffle+Fletcher32 chunk kernels
// (mc_fletcher.hip).
#pragma once

#include "mc_common.h"

template <int ES, int QMUL = 1>
struct Geom {
  static constexpr int Q = (ES >= 16 ? 2 : 4) * QMUL;  // quads per thread per tile
  static constexpr int TE = Q * 4 * MC_BLOCK;       // elements per tile
  static constexpr int TB = TE * ES;                // bytes per tile (either side)
  static constexpr int NV = TB / 16 / MC_BLOCK;     // 16-B units per thread per tile
  static constexpr int PU = TE / 16;                // 16-B units per plane per tile
};

struct ChunkMap {
  size_t count;            // elements per chunk
  size_t tiles_per_chunk;  // full tiles per chunk
  size_t src_stride;       // bytes between chunks (source)
  size_t dst_stride;       // bytes between chunks (destination)
  unsigned group;          // consecutive tiles a block takes per grid-stride step
};

// Tile schedule: tiles are taken in groups of m.group consecutive tiles, groups
// grid-strided over the blocks (group = 1 is a plain grid-stride loop).
#define MC_FOR_TILES(tile, ntiles, m)                                               \
  for (size_t _g = blockIdx.x; _g * (m).group < (ntiles); _g += gridDim.x)          \
    for (size_t tile = _g * (m).group, _e = min((ntiles), tile + (m).group); tile < _e; ++tile)

// load / store the es dwords of one quad (16-B accesses where possible);
// NT selects nontemporal global accesses, LDS accesses use NT = false.
template <int ES, bool NT>
MC_DEV void load_quad(const uint8_t *p, uint32_t (&w)[ES]) {
  if constexpr (ES == 2) {
    const mc_u32x2 v = mc_ld8<NT>(p);
    w[0] = v.x; w[1] = v.y;
  } else {
#pragma unroll
    for (int k = 0; k < ES / 4; ++k) {
      const mc_u32x4 v = mc_ld16<NT>(p + 16 * k);
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
  }
}

template <int ES, bool NT>
MC_DEV void store_quad(uint8_t *p, const uint32_t (&w)[ES]) {
  if constexpr (ES == 2) {
    mc_st8<NT>(p, mc_u32x2{w[0], w[1]});
  } else {
#pragma unroll
    for (int k = 0; k < ES / 4; ++k)
      mc_st16<NT>(p + 16 * k, mc_u32x4{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]});
  }
}

// Shared driver of every shuffle entry point (mc_shuffle.hip), also used by
// the fused Shuffle+Fletcher32 ops: variant 0 = the measured default schedule
// (the other layouts exist for the lab's sweeps, tools/lab); br != NULL fuses
// BitRound into the encode.
int mc_shuffle_impl(const void *src, size_t src_stride, void *dst, size_t dst_stride, size_t nchunks,
                    size_t chunk_bytes, size_t es, bool enc, int variant, int max_blocks, const McBitRound *br,
                    hipStream_t st);
