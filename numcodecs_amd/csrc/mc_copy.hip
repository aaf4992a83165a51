// mc_copy.hip -- device-to-device copies of rows of bytes (1-D: one row).
//
// The pass-through cases of the codecs are plain copies: Shuffle with
// elementsize <= 1 (shuffle.py:31-33), AsType to the same dtype, a decode
// into a caller's `out` (compat.py ndarray_copy), Jenkins' payload copy,
// Blosc blocks left unfiltered.  hipMemcpyAsync DtoD streams at ~4.5 TB/s
// on MI355X; the same 16-B nontemporal lane-contiguous pattern as the codec
// kernels reaches the ~6.4 TB/s copy ceiling (bench.py roofline.achievable).
// Tiles of U * 256 16-B vectors, every load of a tile issued before any of
// its stores, workgroups striding over the tiles (grid cap); rows whose addresses are only 4-B aligned use dwordx4 accesses
// at dword alignment; anything less aligned goes to hipMemcpy2DAsync.
#include "mc_common.h"

#include <stdlib.h>

namespace {

template <int AL>
MC_DEV mc_u32x4 cp_ld(const uint8_t *p) {
  if constexpr (AL == 2) {
    return mc_ld16<true>(p);
  } else {
    mc_u32x4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), 16);
    return v;
  }
}
template <int AL>
MC_DEV void cp_st(uint8_t *p, mc_u32x4 v) {
  if constexpr (AL == 2) mc_st16<true>(p, v);
  else __builtin_memcpy(__builtin_assume_aligned(p, 4), &v, 16);
}

// tile = U * MC_BLOCK vectors of one row; workgroups stride over the tiles
template <int AL, int U>
__global__ __launch_bounds__(MC_BLOCK) void k_copy_rows(const uint8_t *__restrict__ src, size_t ss,
                                                         uint8_t *__restrict__ dst, size_t ds,
                                                         size_t width, size_t tiles_per_row,
                                                         size_t total_tiles) {
  constexpr size_t TILE_VECS = (size_t)U * MC_BLOCK;
  const size_t nvec = width / 16;
  for (size_t tile = blockIdx.x; tile < total_tiles; tile += gridDim.x) {
    const size_t row = tile / tiles_per_row;
    const size_t t = tile - row * tiles_per_row;
    const uint8_t *s = src + row * ss;
    uint8_t *d = dst + row * ds;
    const size_t v0 = t * TILE_VECS + threadIdx.x;
    mc_u32x4 v[U];
    if ((t + 1) * TILE_VECS <= nvec) {
      // a whole tile: every load issued before any store, no per-vector test
      // (the tested form let the compiler interleave them: 5.95 against
      // 6.36 TB/s for the plain calibration copy, tools/lab/lab_bw.hip)
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = cp_ld<AL>(s + (v0 + u * MC_BLOCK) * 16);
#pragma unroll
      for (int u = 0; u < U; ++u) cp_st<AL>(d + (v0 + u * MC_BLOCK) * 16, v[u]);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v0 + u * MC_BLOCK < nvec) v[u] = cp_ld<AL>(s + (v0 + u * MC_BLOCK) * 16);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v0 + u * MC_BLOCK < nvec) cp_st<AL>(d + (v0 + u * MC_BLOCK) * 16, v[u]);
    }
    if (t == tiles_per_row - 1)  // the last width % 16 bytes of the row
      for (size_t b = nvec * 16 + threadIdx.x; b < width; b += MC_BLOCK) d[b] = s[b];
  }
}

inline int copy_align(const void *p, size_t stride, size_t rows) {
  const uintptr_t a = (uintptr_t)p | (rows > 1 ? stride : 0);
  return a % 16 == 0 ? 2 : a % 4 == 0 ? 1 : 0;
}

// schedule (mc_sched.h): copy_u = vectors per thread per tile (4 or 8),
// copy_grid = workgroup cap (0 = one tile per workgroup).  Defaults from
// profiles/r01/copy_knobs_ab.jsonl: 16 KiB tiles, one per workgroup,
// 5.7-5.9 TB/s against 4.7-5.3 TB/s for hipMemcpyAsync DtoD (256 MiB, 1 GiB).
inline int copy_u() { return mc_sched.copy_u == 8 ? 8 : 4; }
inline size_t copy_grid_cap() {
  return mc_sched.copy_grid > 0 ? (size_t)mc_sched.copy_grid : (size_t)0x7fffffff;
}

template <int AL, int U>
void launch_copy(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t width, size_t rows,
                 size_t tpr, hipStream_t st) {
  const size_t total = tpr * rows;
  const size_t cap = copy_grid_cap();
  const unsigned grid = (unsigned)(total < cap ? total : cap);
  k_copy_rows<AL, U><<<grid, MC_BLOCK, 0, st>>>(s, ss, d, ds, width, tpr, total);
}

}  // namespace

// shared with the other translation units (mc_common.h)
int mc_copy_rows_impl(const void *src, size_t src_stride, void *dst, size_t dst_stride, size_t width,
                      size_t rows, hipStream_t st) {
  if (width == 0 || rows == 0) return MC_OK;
  if (rows == 1) src_stride = dst_stride = width;
  int al = copy_align(src, src_stride, rows);
  const int ad = copy_align(dst, dst_stride, rows);
  al = al < ad ? al : ad;
  if (al == 0) {
    if (rows == 1) return mc_hip_status(hipMemcpyAsync(dst, src, width, hipMemcpyDeviceToDevice, st));
    return mc_hip_status(
        hipMemcpy2DAsync(dst, dst_stride, src, src_stride, width, rows, hipMemcpyDeviceToDevice, st));
  }
  const int U = copy_u();
  const size_t tile = (size_t)U * MC_BLOCK;
  const size_t tpr = width / 16 >= 1 ? (width / 16 + tile - 1) / tile : 1;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  if (al == 2) {
    if (U == 8) launch_copy<2, 8>(s, src_stride, d, dst_stride, width, rows, tpr, st);
    else launch_copy<2, 4>(s, src_stride, d, dst_stride, width, rows, tpr, st);
  } else {
    if (U == 8) launch_copy<1, 8>(s, src_stride, d, dst_stride, width, rows, tpr, st);
    else launch_copy<1, 4>(s, src_stride, d, dst_stride, width, rows, tpr, st);
  }
  return mc_last_launch();
}

extern "C" {

int mc_copy(const void *src, void *dst, size_t nbytes, mc_stream_t stream) {
  if (nbytes && (!src || !dst)) return MC_EINVAL;
  return mc_copy_rows_impl(src, nbytes, dst, nbytes, nbytes, 1, (hipStream_t)stream);
}

int mc_copy_rows(const void *src, size_t src_stride, void *dst, size_t dst_stride, size_t width,
                 size_t rows, mc_stream_t stream) {
  if (rows == 0 || width == 0) return MC_OK;
  if (!src || !dst || (rows > 1 && (src_stride < width || dst_stride < width))) return MC_EINVAL;
  return mc_copy_rows_impl(src, src_stride, dst, dst_stride, width, rows, (hipStream_t)stream);
}

}  // extern "C"
