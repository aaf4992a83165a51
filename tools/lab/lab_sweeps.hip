// lab_sweeps.hip -- LAB ONLY (libmcodec_lab.so; never part of libmcodec.so or
// include/mcodec.h): explicit-schedule entry points used by the measurement
// sweeps (tools/probe_enc.py, tools/gpu_probe.py, tools/probe_delta.py) and by
// the tests that keep every schedule byte-identical to the default
// (tests/test_gpu_sweep.py).
#include "mc_shuffle.h"

int mc_delta_decode_batch_impl(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                               size_t nchunks, size_t n, int astype, int dtype, int variant,
                               mc_stream_t stream);

size_t mc_delta_dec1p_state_bytes(size_t n, int es);
size_t mc_c4_dec1p_state_bytes(size_t n, int astype);
int mc_delta_dec1p(const void *src, void *dst, size_t n, int es, void *state, hipStream_t st, unsigned spins,
                   uint64_t *trace);
int mc_c4_dec1p(const void *src, void *dst, size_t n, int astype, int dtype, double scale, double offset,
                void *state, hipStream_t st, unsigned spins, uint64_t *trace);

extern "C" {

// The single-pass decodes (lab_scan1p.hip) with an explicit look-back spin
// bound (MC_LB_WAVE_SPINS = 16384 normally; 0 makes every partition whose
// predecessors have not all published yet take the data-derived prefix, the
// guard path).  `state`: mc_lab_*_dec1p_state_bytes() device bytes, zero
// before the first call, left zero by every call.
// `trace` (may be NULL): 8 uint64 per partition, wall_clock64() at ticket,
// staged, look-back resolved, emit start, emitted, and the workgroup id.
size_t mc_lab_delta_dec1p_state_bytes(size_t n, int es) { return mc_delta_dec1p_state_bytes(n, es); }
size_t mc_lab_c4_dec1p_state_bytes(size_t n, int astype) { return mc_c4_dec1p_state_bytes(n, astype); }

int mc_lab_delta_dec1p(const void *src, void *dst, size_t n, int es, void *state, unsigned spins,
                       uint64_t *trace, mc_stream_t stream) {
  return mc_delta_dec1p(src, dst, n, es, state, (hipStream_t)stream, spins, trace);
}

int mc_lab_c4_dec1p(const void *src, void *dst, size_t n, int astype, int dtype, double scale, double offset,
                    void *state, unsigned spins, uint64_t *trace, mc_stream_t stream) {
  return mc_c4_dec1p(src, dst, n, astype, dtype, scale, offset, state, (hipStream_t)stream, spins, trace);
}

// Shuffle with an explicit kernel layout and grid (mc_shuffle.hip Variant):
// bits 0-2 layout (0 default, 1 register/dword stores, 2 LDS-staged 16-B
// stores, 3 LDS both sides, 4 generic byte kernel, 5 lane pairs), | 8
// temporal accesses, | 16 / | 128 2x / 4x tiles, bits 5-6 tile group,
// | 256 software-pipelined persistent loop, | 512 8x tiles.  max_blocks 0 =
// one workgroup per tile, the product's grid for large buffers (round 4:
// until then 0 capped an explicit layout at MC_MAX_GRID = 2048 workgroups,
// which made every layout with more than 2048 tiles loop and measure slower
// than it runs in the product); < 0 = that 2048 cap; > 0 = this cap.
static int lab_grid_cap(int max_blocks) {
  return max_blocks == 0 ? 0x7fffffff : max_blocks < 0 ? (int)MC_MAX_GRID : max_blocks;
}

int mc_lab_shuffle_variant(const void *src, void *dst, size_t nbytes, size_t elementsize, int encode,
                           int variant, int max_blocks, mc_stream_t stream) {
  if (variant < 0 || (variant & ~0x3FF) != 0) return MC_EINVAL;
  max_blocks = lab_grid_cap(max_blocks);
  return mc_shuffle_impl(src, 0, dst, 0, 1, nbytes, elementsize, encode != 0, variant, max_blocks, nullptr,
                         (hipStream_t)stream);
}

// a batch of nchunks rows (row strides ss / ds bytes) with an explicit
// layout, as mc_lab_shuffle_variant
int mc_lab_shuffle_batch_variant(const void *src, size_t ss, void *dst, size_t ds, size_t nchunks, size_t nbytes,
                                 size_t elementsize, int encode, int variant, int max_blocks, mc_stream_t stream) {
  if (variant < 0 || (variant & ~0x3FF) != 0) return MC_EINVAL;
  max_blocks = lab_grid_cap(max_blocks);
  return mc_shuffle_impl(src, ss, dst, ds, nchunks, nbytes, elementsize, encode != 0, variant, max_blocks, nullptr,
                         (hipStream_t)stream);
}

// BitRound fused into the Shuffle encode (mc_bitround_shuffle) with an
// explicit layout, as mc_lab_shuffle_variant.
int mc_lab_bitround_shuffle_variant(const void *src, void *dst, size_t n, int itemsize, int keepbits,
                                    int variant, int max_blocks, mc_stream_t stream) {
  if (variant < 0 || (variant & ~0x3FF) != 0) return MC_EINVAL;
  if (!(itemsize == 2 || itemsize == 4 || itemsize == 8)) return MC_EINVAL;
  const int mbits = itemsize == 2 ? 10 : itemsize == 4 ? 23 : 52;
  if (keepbits < 0 || keepbits >= mbits) return MC_EINVAL;
  const McBitRound br = mc_make_bitround(itemsize, keepbits);
  max_blocks = lab_grid_cap(max_blocks);
  return mc_shuffle_impl(src, 0, dst, 0, 1, n * (size_t)itemsize, (size_t)itemsize, true, variant, max_blocks, &br,
                         (hipStream_t)stream);
}

// mc_delta_decode_batch with an explicit float-chain schedule (LDS slot
// bytes / chain values per LDS read group): 0 default (by batch size),
// 1 32 KiB/16, 2 32 KiB/32, 3 8 KiB/16, 4 8 KiB/32, 5 4 KiB/32.  Integer
// dtypes ignore it.  All give identical bytes.
int mc_lab_delta_decode_batch_variant(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                                      size_t nchunks, size_t n, int astype, int dtype, int variant,
                                      mc_stream_t stream) {
  return mc_delta_decode_batch_impl(src, src_stride, dst, dst_stride, nchunks, n, astype, dtype, variant,
                                    stream);
}

}  // extern "C"
