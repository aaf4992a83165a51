// lab_bw.hip -- LAB ONLY (libmcodec_lab.so): the HBM copy calibration that
// bench.py's roofline "copy ceiling" and the Shuffle sweeps compare against.
// A plain 16-B/lane copy, U vectors per thread per tile with every load of
// a tile issued before its stores, workgroups striding over the tiles
// (`grid`, 0 = one tile per workgroup), nontemporal loads and/or stores.
// Not a codec: it moves bytes unchanged, whole tiles only.
#include "mc_common.h"

namespace {

template <int U, bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(MC_BLOCK) void k_lab_bw_copy(const mc_u32x4 *__restrict__ s, mc_u32x4 *__restrict__ d,
                                                         size_t tiles) {
  for (size_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const size_t base = t * U * MC_BLOCK + threadIdx.x;
    mc_u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = mc_ld16<NT_LD>(s + base + u * MC_BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) mc_st16<NT_ST>(d + base + u * MC_BLOCK, v[u]);
  }
}

template <int U>
int launch_bw(const mc_u32x4 *s, mc_u32x4 *d, size_t tiles, unsigned grid, int nt, hipStream_t st) {
  switch (nt) {
    case 0: k_lab_bw_copy<U, false, false><<<grid, MC_BLOCK, 0, st>>>(s, d, tiles); break;
    case 1: k_lab_bw_copy<U, true, false><<<grid, MC_BLOCK, 0, st>>>(s, d, tiles); break;
    case 2: k_lab_bw_copy<U, false, true><<<grid, MC_BLOCK, 0, st>>>(s, d, tiles); break;
    default: k_lab_bw_copy<U, true, true><<<grid, MC_BLOCK, 0, st>>>(s, d, tiles); break;
  }
  return mc_last_launch();
}

}  // namespace

// nt: bit 0 = nontemporal loads, bit 1 = nontemporal stores.  nbytes must be
// a whole number of tiles (U * 4 KiB).
extern "C" int mc_lab_bw_copy(const void *src, void *dst, size_t nbytes, int u, int grid, int nt,
                              mc_stream_t stream) {
  if (!src || !dst || (u != 1 && u != 2 && u != 4 && u != 8) || grid < 0 || nt < 0 || nt > 3) return MC_EINVAL;
  const size_t tb = (size_t)u * MC_BLOCK * 16;
  if (nbytes == 0 || nbytes % tb || (uintptr_t)src % 16 || (uintptr_t)dst % 16) return MC_EINVAL;
  const size_t tiles = nbytes / tb;
  const unsigned g = grid == 0 || (size_t)grid > tiles ? (unsigned)tiles : (unsigned)grid;
  const mc_u32x4 *s = static_cast<const mc_u32x4 *>(src);
  mc_u32x4 *d = static_cast<mc_u32x4 *>(dst);
  hipStream_t st = (hipStream_t)stream;
  switch (u) {
    case 1: return launch_bw<1>(s, d, tiles, g, nt, st);
    case 2: return launch_bw<2>(s, d, tiles, g, nt, st);
    case 4: return launch_bw<4>(s, d, tiles, g, nt, st);
    default: return launch_bw<8>(s, d, tiles, g, nt, st);
  }
}
