/*
 * mcodec.h -- C ABI of libmcodec.so, the MI355X (gfx950) kernels behind
 * numcodecs_amd.
 *
 * This is the drop-in boundary for numcodecs' per-element filter codecs and
 * its Fletcher32 checksum.  Every entry point takes plain device pointers,
 * byte/element counts and a hipStream_t (passed as `mc_stream_t`, NULL = the
 * legacy default stream).  Entry points never allocate device memory, never
 * synchronise the stream and never throw: they enqueue kernels and return a
 * status (MC_OK, a negative MC_E* code, or MC_EHIP_BASE - hipError_t).
 * Argument checks that numcodecs reports as Python exceptions are done by the
 * host layer (the numcodecs_amd Python modules) before the call; the library re-checks what
 * it needs for memory safety and returns MC_EINVAL.
 *
 * Reference interface each entry point replaces (paths relative to the
 * numcodecs source tree, src/numcodecs/):
 *   mc_shuffle / mc_unshuffle ...... _shuffle.pyx:11-18 _doShuffle / :23-30 _doUnshuffle
 *                                    (called from shuffle.py:40-58 Shuffle.encode/decode)
 *   mc_bitround .................... bitround.py:45-69 BitRound.encode (numpy int ops)
 *   mc_bitround_shuffle ............ bitround.py:45-69 followed by _shuffle.pyx:11-18, fused
 *   mc_delta_encode ................ delta.py:52-67 Delta.encode (np.diff)
 *   mc_delta_decode ................ delta.py:69-83 Delta.decode (np.cumsum)
 *   mc_fso_encode / mc_fso_decode .. fixedscaleoffset.py:83-97 / :99-113
 *   mc_quantize .................... quantize.py:60-76 Quantize.encode
 *   mc_cast ........................ ndarray.astype as used by quantize.py:76,80,
 *                                    fixedscaleoffset.py:97,110, compat.py:177-206
 *   mc_fletcher32* ................. fletcher32.pyx:24-57 _fletcher32, :75-89 encode,
 *                                    :91-115 decode; _utils.pxd:11-24 store/load_le32
 *   mc_checksum32_batch /
 *   mc_checksum32_encode_batch /
 *   mc_checksum32_decode_batch ..... checksum32.py:45-88 Checksum32.encode/decode with
 *                                    CRC32 (:95-111, zlib.crc32), Adler32 (:114-130,
 *                                    zlib.adler32), CRC32C (:189-209), JenkinsLookup3
 *                                    (:133-181 over jenkins.pyx:93-325)
 *   mc_packbits / mc_unpackbits .... packbits.py:33-82 PackBits.encode/decode
 *   mc_blosc_filter ................ blosc.pyx:67-71,211-326 SHUFFLE / BITSHUFFLE as
 *                                    c-blosc applies them per block (shuffle.c)
 *   *_batch ........................ no reference counterpart: the Zarr caller loops
 *                                    Codec.encode per chunk; these run B equal-size
 *                                    chunks in one launch (chunk b at base + b*stride).
 */
#ifndef MCODEC_H
#define MCODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *mc_stream_t; /* hipStream_t */

#define MC_ABI_VERSION 2

/* status codes */
#define MC_OK 0
#define MC_EINVAL (-22)      /* bad argument (size, dtype, alignment, NULL) */
#define MC_ENOSPC (-28)      /* workspace too small */
#define MC_EPROTO (-71)      /* a stream ended without publishing its verdict */

/* Size in uint32 words of the arrival counter (`ticket`) that the one-launch
 * verifies take: 64 shard words on separate 128-B lines plus a top word. */
#define MC_ARRIVAL_WORDS 2080
#define MC_EHIP_BASE (-1000) /* MC_EHIP_BASE - (int)hipError_t */

/* dtype codes (numpy kind + itemsize).  A code names the little-endian
 * (native) dtype; MC_BIG_ENDIAN OR'd into the code of a multi-byte dtype
 * names the same dtype stored big-endian ('>i2', '>f4', ... -- numpy's
 * non-native byte order, as Zarr v2 arrays converted from netCDF/HDF5 carry
 * it).  Byte order only changes how an element sits in memory: the kernels
 * reverse its bytes in registers on load / before the store and compute
 * exactly as for the little-endian dtype (delta.py:52-83,
 * fixedscaleoffset.py:83-113, quantize.py:60-82 and astype.py:46-58 compute
 * big-endian arrays through numpy the same way).  Compute dtypes (the t1..t4
 * of the FixedScaleOffset entry points) are never big-endian: numpy's
 * arithmetic results are native. */
#define MC_BIG_ENDIAN 32
enum mc_dtype {
  MC_B1 = 0, /* '|b1' bool */
  MC_I1 = 1, /* '|i1' */
  MC_I2 = 2, /* '<i2' */
  MC_I4 = 3, /* '<i4' */
  MC_I8 = 4, /* '<i8' */
  MC_U1 = 5, /* '|u1' */
  MC_U2 = 6, /* '<u2' */
  MC_U4 = 7, /* '<u4' */
  MC_U8 = 8, /* '<u8' */
  MC_F2 = 9, /* '<f2' */
  MC_F4 = 10, /* '<f4' */
  MC_F8 = 11, /* '<f8' */
  MC_NDTYPES = 12,
  /* extended dtypes (round 5): accepted by mc_cast / mc_cast_units,
   * mc_delta_encode / mc_delta_decode (single chunk) and the FixedScaleOffset
   * entry points; the batched and fused entry points refuse them (MC_EINVAL). */
  MC_C8 = 12,  /* '<c8'  complex64: two f4 components (real, imag) */
  MC_C16 = 13, /* '<c16' complex128: two f8 components */
  MC_TD8 = 14, /* '<m8[unit]' timedelta64: int64 ticks, NaT = INT64_MIN */
  MC_DT8 = 15, /* '<M8[unit]' datetime64: int64 ticks, NaT = INT64_MIN */
  /* round 6: numpy's longdouble on x86-64 -- the x87 80-bit extended format
   * (64-bit significand with explicit integer bit, 15-bit exponent) stored in
   * 16 bytes, 6 of them padding (written as zero; numpy leaves them as
   * whatever the output buffer held, so only the 10 value bytes are numpy's).
   * Every operation is one x87 operation: round to nearest even at 64 bits,
   * gradual underflow, x87 NaN rules (a QNaN beats an SNaN, else the larger
   * significand; SNaNs quieted), the "real indefinite" NaN for invalid
   * operations and for the encodings x87 rejects (unnormals, pseudo-NaNs /
   * pseudo-infinities); casts as gcc compiles numpy's C casts (fst m32 / m64,
   * fistp with truncation, float16 through float32). */
  MC_F16L = 16, /* '<f16' longdouble */
  MC_C32 = 17,  /* '<c32' clongdouble: two MC_F16L components */
  MC_NDTYPES_EXT = 18
};

int mc_abi_version(void);
const char *mc_strerror(int status);
/* number of HIP devices visible to the runtime the library is bound to */
int mc_device_count(void);

/* Device-to-device copy (the codecs' pass-through cases: Shuffle with
 * elementsize <= 1, shuffle.py:31-33; AsType to the same dtype; decode into
 * `out`, compat.py:173-206 ndarray_copy): nbytes from src to dst, or `rows`
 * rows of `width` bytes at src + r*src_stride -> dst + r*dst_stride.  src
 * and dst must not overlap. */
int mc_copy(const void *src, void *dst, size_t nbytes, mc_stream_t stream);
int mc_copy_rows(const void *src, size_t src_stride, void *dst,
                 size_t dst_stride, size_t width, size_t rows,
                 mc_stream_t stream);

/* ---- Shuffle ---------------------------------------------------------- */
/* Byte transpose of the (nbytes/elementsize, elementsize) byte matrix:
 *   dst[b*count + i] = src[i*elementsize + b],  count = nbytes/elementsize.
 * nbytes % elementsize must be 0; elementsize >= 1 (1 is a plain copy).
 * src and dst must not overlap. */
int mc_shuffle(const void *src, void *dst, size_t nbytes, size_t elementsize,
               mc_stream_t stream);
/* Inverse: dst[i*elementsize + b] = src[b*count + i]. */
int mc_unshuffle(const void *src, void *dst, size_t nbytes, size_t elementsize,
                 mc_stream_t stream);
/* Batched: nchunks independent chunks of chunk_bytes each; chunk c is read at
 * src + c*src_stride and written at dst + c*dst_stride (strides in bytes). */
int mc_shuffle_batch(const void *src, size_t src_stride, void *dst,
                     size_t dst_stride, size_t nchunks, size_t chunk_bytes,
                     size_t elementsize, mc_stream_t stream);
int mc_unshuffle_batch(const void *src, size_t src_stride, void *dst,
                       size_t dst_stride, size_t nchunks, size_t chunk_bytes,
                       size_t elementsize, mc_stream_t stream);

/* ---- BitRound --------------------------------------------------------- */
/* n elements of itemsize 2 (f16), 4 (f32) or 8 (f64); 0 <= keepbits < max
 * mantissa bits (10/23/52).  dst receives the rounded bit patterns. */
int mc_bitround(const void *src, void *dst, size_t n, int itemsize,
                int keepbits, mc_stream_t stream);
/* BitRound then Shuffle(elementsize=itemsize) in one pass (dst = shuffled). */
int mc_bitround_shuffle(const void *src, void *dst, size_t n, int itemsize,
                        int keepbits, mc_stream_t stream);

/* ---- Delta ------------------------------------------------------------ */
/* dst[0] = astype(src[0]); dst[i] = astype(src[i] - src[i-1]) computed in
 * dtype (bool: src[i] != src[i-1]).  n >= 1.
 * Extended dtypes: complex differences per component; timedelta / datetime
 * differences are timedelta ticks with NaT propagation (NaT if either side
 * is NaT, else the wrap-around difference), then cast to astype as
 * mc_cast does (same unit). */
int mc_delta_encode(const void *src, void *dst, size_t n, int dtype,
                    int astype, mc_stream_t stream);
/* dst = cumsum(dtype(src)) accumulated in dtype (bool: logical or).  Integer
 * dtypes use a parallel scan (modular arithmetic, bit-exact); float dtypes
 * keep numpy's sequential left-to-right rounding.  For f4/f8 with astype ==
 * dtype, 16-B aligned buffers and the workspace this function asks for, a
 * parallel scan is verified element by element against that recurrence and
 * the serial chain reruns from the first mismatch (bit-exact for any data;
 * smooth data verify entirely).  Otherwise (or with no workspace) float
 * decode is the serial chain.  The workspace's last 8 bytes hold the index
 * of the first mismatch (n if none) after the call.
 * Extended dtypes (the workspace is then required, MC_ENOSPC without it):
 *  - dtype MC_TD8 from astype MC_TD8 / an integer / bool: numpy's timedelta
 *    add loop -- the wrap-around prefix sum up to the first element that is
 *    NaT or whose running sum is INT64_MIN, NaT from there on (an integer
 *    scan plus a NaT pass); dtype MC_I8 from astype MC_TD8 likewise.
 *  - complex dtype or astype: per component, the running sums of the real
 *    and imaginary parts in the component type of promote(astype, dtype)
 *    (each one mc_delta_decode of a real plane, so float speculation and
 *    the serial chain apply per component), cast to dtype. */
size_t mc_delta_decode_workspace(size_t n, int astype, int dtype);
/* `ticket`: MC_ARRIVAL_WORDS device words (8-B aligned), zero before the
 * first call and left zero (one per stream): same-width integer decodes of
 * 1/2/4-byte elements run as two launches (tile-total scan folded into the
 * passes); NULL: the three-pass scan.  Same bytes either way. */
int mc_delta_decode(const void *src, void *dst, size_t n, int astype,
                    int dtype, void *workspace, size_t workspace_bytes,
                    uint32_t *ticket, mc_stream_t stream);
/* Batched Delta over nchunks chunks of n elements each (chunk c read at
 * src + c*src_stride, written at dst + c*dst_stride; strides in bytes).
 * Each chunk is an independent Delta (its own first element / cumsum).
 * Decode runs one workgroup per chunk (integer: single-pass scan with a
 * running carry; float: one sequential add chain per chunk) and needs no
 * workspace. */
/* mc_delta_decode_batch with a workspace (mc_delta_decode_batch_workspace
 * bytes: 8 per chunk for f4/f8 with astype == dtype, else 0).  f4/f8 chunks
 * (16-B aligned buffers and strides) then decode by the verified
 * speculative scan of mc_delta_decode, one workgroup per chunk, and chunks
 * with a rounding mismatch finish as a serial chain from the start of the
 * 16 KiB tile holding it (bit-exact for any data); workspace[c] = that
 * element index (n if the chunk verified entirely).  Every
 * other case, or no workspace, is mc_delta_decode_batch. */
size_t mc_delta_decode_batch_workspace(size_t nchunks, size_t n, int astype,
                                       int dtype);
int mc_delta_decode_batch_ws(const void *src, size_t src_stride, void *dst,
                             size_t dst_stride, size_t nchunks, size_t n,
                             int astype, int dtype, void *workspace,
                             size_t workspace_bytes, mc_stream_t stream);
int mc_delta_encode_batch(const void *src, size_t src_stride, void *dst,
                          size_t dst_stride, size_t nchunks, size_t n,
                          int dtype, int astype, mc_stream_t stream);
int mc_delta_decode_batch(const void *src, size_t src_stride, void *dst,
                          size_t dst_stride, size_t nchunks, size_t n,
                          int astype, int dtype, mc_stream_t stream);

/* ---- FixedScaleOffset / Quantize / casts ------------------------------ */
/* Scalars arrive already converted (on the host, by numpy's NEP 50 rules) to
 * the compute dtype of the operation that uses them: *_f for float compute
 * dtypes, *_i for integer compute dtypes.
 * encode: dst = astype(rint((dtype(x) -[t1] offset) *[t2] scale)) */
int mc_fso_encode(const void *src, void *dst, size_t n, int dtype, int t1,
                  int t2, int astype, double offset_f, int64_t offset_i,
                  double scale_f, int64_t scale_i, mc_stream_t stream);
/* decode: dst = dtype((astype(x) /[t3] scale) +[t4] offset); t3, t4 float */
int mc_fso_decode(const void *src, void *dst, size_t n, int astype, int t3,
                  int t4, int dtype, double scale, double offset,
                  mc_stream_t stream);
/* Quantize encode: dst = astype(rint(scale *[dtype] x) /[dtype] scale) */
int mc_quantize(const void *src, void *dst, size_t n, int dtype, int astype,
                double scale, mc_stream_t stream);
/* numpy `astype` (unsafe casting; x86-64 results for out-of-range/NaN
 * float->int, correctly rounded float narrowing). */
int mc_cast(const void *src, void *dst, size_t n, int from_dtype,
            int to_dtype, mc_stream_t stream);

/* ---- extended dtypes: complex64/128, timedelta64, datetime64 ------------- */
/* The codes carry no datetime unit: ticks are int64 in the caller's unit.
 * numpy astype semantics (astype.py:46-58):
 *  - complex -> complex: per-component float cast; complex -> bool: re != 0
 *    or im != 0; complex -> other real: the real part cast (numpy's
 *    ComplexWarning is the host's business); real -> complex: (x, +0).
 *  - timedelta/datetime <-> int/float/bool/complex: the int64 ticks as an i8
 *    (NaT is INT64_MIN like any other value; float -> ticks truncates with
 *    x86-64 cvttsd2si, NaN/out of range -> INT64_MIN = NaT).
 *  - time -> time: bits, or, with (num, den) != (1, 1) -- numpy's unit
 *    conversion factor of a same-kind cast (m8 -> m8, M8 -> M8 between
 *    linear units; the host computes it) -- NaT kept, else
 *    v*num/den for v >= 0 and (v*num - (den - 1))/den for v < 0 (int64
 *    wrap-around products, C division), as numpy's datetime cast loop does.
 * mc_cast(...) == mc_cast_units(..., 1, 1). */
int mc_cast_units(const void *src, void *dst, size_t n, int from_dtype,
                  int to_dtype, int64_t num, int64_t den, mc_stream_t stream);
/* FixedScaleOffset with complex compute dtypes (fixedscaleoffset.py:83-113):
 * as mc_fso_encode / mc_fso_decode with complex scalars (re, im); integer
 * compute dtypes take offset_i / scale_i.  Complex subtract/add are
 * per component, multiply is (ar*br - ai*bi, ar*bi + ai*br) and divide is
 * numpy's Smith-style loop (umath loops.c.src @TYPE@_divide), every scalar
 * op rounded in the component type with x86-64 NaN propagation; rint per
 * component.  The real entry points accept these codes too (imag parts 0). */
int mc_fso_encode_x(const void *src, void *dst, size_t n, int dtype, int t1,
                    int t2, int astype, double offset_re, double offset_im,
                    int64_t offset_i, double scale_re, double scale_im,
                    int64_t scale_i, mc_stream_t stream);
int mc_fso_decode_x(const void *src, void *dst, size_t n, int astype, int t3,
                    int t4, int dtype, double scale_re, double scale_im,
                    double offset_re, double offset_im, mc_stream_t stream);
/* FixedScaleOffset with the scalars given as raw bytes (host memory, read
 * during the call): `offset` / `scale` hold the value numpy computes with, in
 * the compute dtype t1 / t2 (encode) or scale in t3 / offset in t4 (decode),
 * native byte order, x_itemsize bytes (16 for MC_F16L, 32 for MC_C32).  Any
 * dtype code; required when a longdouble value does not fit a double
 * (fixedscaleoffset.py:83-113 with '<f16' / '<c32'). */
int mc_fso_encode_raw(const void *src, void *dst, size_t n, int dtype, int t1,
                      int t2, int astype, const void *offset, const void *scale,
                      mc_stream_t stream);
int mc_fso_decode_raw(const void *src, void *dst, size_t n, int astype, int t3,
                      int t4, int dtype, const void *scale, const void *offset,
                      mc_stream_t stream);
/* numpy's calendar datetime64 cast (astype.py:46-58 between datetime64 units
 * where one side is years or months and the other is not: numpy's
 * datetimestruct path, datetime.c convert_datetime_to_datetimestruct /
 * convert_datetimestruct_to_datetime): ticks * src_num in unit src_unit ->
 * the proleptic Gregorian date -> dst_unit ticks floor-divided by dst_num;
 * NaT stays NaT.  Units are numpy's NPY_DATETIMEUNIT codes (0 Y, 1 M, 2 W,
 * 3 D, 4 h, 5 m, 6 s, 7 ms, 8 us, 9 ns, 10 ps, 11 fs, 12 as). */
int mc_cast_calendar(const void *src, void *dst, size_t n, int from_dtype,
                     int to_dtype, int src_unit, int64_t src_num, int dst_unit,
                     int64_t dst_num, mc_stream_t stream);

/* ---- Fletcher32 ------------------------------------------------------- */
size_t mc_fletcher32_workspace(size_t nbytes);
/* *out_sum (device) = fletcher32(src[0:nbytes]); nbytes >= 0. */
int mc_fletcher32(const void *src, size_t nbytes, uint32_t *out_sum,
                  void *workspace, size_t workspace_bytes, mc_stream_t stream);
/* dst[0:nbytes] = src; dst[nbytes:nbytes+4] = LE32(fletcher32(src)). */
int mc_fletcher32_encode(const void *src, void *dst, size_t nbytes,
                         void *workspace, size_t workspace_bytes,
                         mc_stream_t stream);
/* mc_fletcher32_encode in ONE launch: the checksum's last blocks fold the
 * partials and write the footer (no finalize kernel).  `ticket` as for
 * mc_fletcher32_verify_fused; NULL = mc_fletcher32_encode.  Workspace:
 * mc_fletcher32_workspace(nbytes).  Replaces fletcher32.pyx:60-85
 * (Fletcher32.encode) for one device chunk. */
int mc_fletcher32_encode_fused(const void *src, void *dst, size_t nbytes,
                               void *workspace, size_t workspace_bytes,
                               uint32_t *ticket, mc_stream_t stream);
/* out_pair (device, 2 words) = {fletcher32(src[0:nbytes-4]),
 * LE32(src[nbytes-4:nbytes])}; nbytes >= 4. */
int mc_fletcher32_verify(const void *src, size_t nbytes, uint32_t *out_pair,
                         void *workspace, size_t workspace_bytes,
                         mc_stream_t stream);
/* mc_fletcher32_verify in ONE launch: the checksum's last blocks fold the
 * partials (no finalize kernel).  `ticket`: MC_ARRIVAL_WORDS device uint32
 * words (an arrival counter, 8-B aligned), zero before the first call and left zero by every call
 * (keep one per stream); NULL = mc_fletcher32_verify (seq must be 0).
 * out_rec = {computed, stored, seq, -}: with seq != 0 the kernel writes
 * out_rec[2] = seq after the verdict, so with out_rec = the device address of
 * an mc_verdict_alloc record the caller waits with mc_verdict_wait (no stream
 * synchronisation, no device-to-host copy); seq == 0 writes words 0-1 only. */
int mc_fletcher32_verify_fused(const void *src, size_t nbytes, uint32_t *out_rec,
                               uint32_t seq, void *workspace, size_t workspace_bytes,
                               uint32_t *ticket, mc_stream_t stream);
/* out_sums[c] = fletcher32(chunk c), chunk c = src + c*stride, chunk_bytes. */
size_t mc_fletcher32_batch_workspace(size_t nchunks, size_t chunk_bytes);
int mc_fletcher32_batch(const void *src, size_t stride, size_t nchunks,
                        size_t chunk_bytes, uint32_t *out_sums,
                        void *workspace, size_t workspace_bytes,
                        mc_stream_t stream);
/* Fletcher32.encode of every chunk: dst row c = chunk c ++ LE32 checksum
 * (dst_stride >= chunk_bytes + 4, chunk_bytes >= 1), one pass.  Workspace:
 * mc_fletcher32_batch_workspace(nchunks, chunk_bytes). */
int mc_fletcher32_encode_batch(const void *src, size_t src_stride, void *dst,
                               size_t dst_stride, size_t nchunks,
                               size_t chunk_bytes, void *workspace,
                               size_t workspace_bytes, mc_stream_t stream);
/* Fletcher32.decode of every encoded row (fletcher32.pyx:91-115): rows of
 * encoded_bytes = payload + LE32 footer.  out_pairs[2c] = fletcher32 of the
 * payload, out_pairs[2c+1] = the stored footer (the caller compares and
 * raises); when dst is not NULL the payloads are compacted into dst rows
 * (dst_stride >= encoded_bytes - 4) in the same pass.  Workspace:
 * mc_fletcher32_batch_workspace(nchunks, encoded_bytes - 4). */
int mc_fletcher32_decode_batch(const void *src, size_t src_stride, void *dst,
                               size_t dst_stride, size_t nchunks,
                               size_t encoded_bytes, uint32_t *out_pairs,
                               void *workspace, size_t workspace_bytes,
                               mc_stream_t stream);

/* ---- fused chunk pipelines (Zarr filter chain -> checksum) ------------- */
/* Workspace for the two calls below. */
size_t mc_shuffle_fletcher32_workspace(size_t nchunks, size_t chunk_bytes,
                                       size_t elementsize);
/* Per chunk: enc = Shuffle(es).encode(chunk) ++ LE32(fletcher32(enc)).
 * dst chunk c at dst + c*dst_stride, dst_stride >= chunk_bytes + 4 (a
 * multiple of 16 keeps the single-pass fused kernel). */
int mc_shuffle_fletcher32_encode_batch(const void *src, size_t src_stride,
                                       void *dst, size_t dst_stride,
                                       size_t nchunks, size_t chunk_bytes,
                                       size_t elementsize, void *workspace,
                                       size_t workspace_bytes,
                                       mc_stream_t stream);
/* Per chunk: verify the footer of src chunk (chunk_bytes + 4 bytes) and
 * unshuffle the payload into dst.  status[2c] = computed checksum,
 * status[2c+1] = stored footer (device array of 2*nchunks words). */
int mc_fletcher32_unshuffle_batch(const void *src, size_t src_stride,
                                  void *dst, size_t dst_stride,
                                  size_t nchunks, size_t chunk_bytes,
                                  size_t elementsize, uint32_t *status,
                                  void *workspace, size_t workspace_bytes,
                                  mc_stream_t stream);

/* Per chunk of n elements: Shuffle(itemsize(astype)).encode(
 *   Delta(astype).encode(FixedScaleOffset(offset, scale, dtype, astype).encode(x)))
 * in one pass (fixedscaleoffset.py:83-97, delta.py:52-67, _shuffle.pyx:11-18).
 * dtype in {F4, F8}; astype in {I2, U2, I4, U4}; n % 16 == 0; 16-B aligned
 * buffers.  offset/scale are the values numpy uses, already converted to
 * dtype (the host checks that numpy computes FSO in dtype, i.e. the scalars
 * are weak Python numbers). */
int mc_fso_delta_shuffle_encode(const void *src, void *dst, size_t n,
                                int dtype, int astype, double offset,
                                double scale, mc_stream_t stream);
/* Inverse chain: unshuffle, cumsum in astype, (x / scale + offset) in
 * float64 cast to dtype (fixedscaleoffset.py:99-113, delta.py:69-83).
 * `ticket`: MC_ARRIVAL_WORDS device words (8-B aligned), zero before the
 * first call and left zero (keep one per stream): the two-launch decode
 * (scan folded into the passes); NULL: the three-pass scan.  Same bytes. */
/* The same chain over nchunks chunks of n elements (Zarr chunk pipelines):
 * chunk c at src + c * src_stride / dst + c * dst_stride (strides 16-B
 * multiples when nchunks > 1).  Encode: one pass (2-D grid of tiles x
 * chunks); decode: a single pass per chunk segment with a running carry --
 * one segment per chunk when nchunks >= 2048, else chunks are cut into
 * segments whose totals a first pass computes (workspace:
 * mc_fso_delta_shuffle_decode_batch_workspace, 0 when not needed).  Same
 * bytes as the single-chunk calls per chunk. */
int mc_fso_delta_shuffle_encode_batch(const void *src, size_t src_stride,
                                      void *dst, size_t dst_stride,
                                      size_t nchunks, size_t n, int dtype,
                                      int astype, double offset, double scale,
                                      mc_stream_t stream);
size_t mc_fso_delta_shuffle_decode_batch_workspace(size_t nchunks, size_t n);
int mc_fso_delta_shuffle_decode_batch(const void *src, size_t src_stride,
                                      void *dst, size_t dst_stride,
                                      size_t nchunks, size_t n, int astype,
                                      int dtype, double scale, double offset,
                                      void *workspace, size_t workspace_bytes,
                                      mc_stream_t stream);
size_t mc_fso_delta_shuffle_decode_workspace(size_t n);
int mc_fso_delta_shuffle_decode(const void *src, void *dst, size_t n,
                                int astype, int dtype, double scale,
                                double offset, void *workspace,
                                size_t workspace_bytes, uint32_t *ticket,
                                mc_stream_t stream);

/* ---- Checksum32 family (checksum32.py:45-209, jenkins.pyx:93-325) ------- */
/* One 32-bit checksum per chunk of a batch (rows at src + c*src_stride):
 *   MC_CK_CRC32    zlib.crc32(chunk, init)              CRC32.checksum
 *   MC_CK_CRC32C   crc32c(chunk, init) (Castagnoli)      CRC32C.checksum
 *   MC_CK_ADLER32  zlib.adler32(chunk, init); the codec passes init = 1.
 *                  Results are reduced mod 65521, equal to zlib for every
 *                  init whose halves are both < 65521 (the codec's 1 is)
 *   MC_CK_JENKINS  jenkins_lookup3(prefix ++ chunk, init); prefix (device
 *                  bytes, may be NULL when prefix_bytes == 0) only here
 * out_sums: device uint32[nchunks].  Workspace from mc_checksum32_workspace
 * (0 for Jenkins, which takes no workspace; pass NULL). */
enum mc_checksum_kind {
  MC_CK_CRC32 = 0,
  MC_CK_CRC32C = 1,
  MC_CK_ADLER32 = 2,
  MC_CK_JENKINS = 3
};
/* where Checksum32.encode puts the LE32 checksum (checksum32.py:48-62) */
enum mc_checksum_location { MC_CK_START = 0, MC_CK_END = 1 };

size_t mc_checksum32_workspace(int kind, size_t nchunks, size_t chunk_bytes);
int mc_checksum32_batch(int kind, const void *src, size_t src_stride,
                        size_t nchunks, size_t chunk_bytes, uint32_t init,
                        const void *prefix, size_t prefix_bytes,
                        uint32_t *out_sums, void *workspace,
                        size_t workspace_bytes, mc_stream_t stream);
/* Checksum32.encode of every chunk: dst row c = checksum (LE32) ++ payload
 * (MC_CK_START) or payload ++ checksum (MC_CK_END); dst_stride >=
 * chunk_bytes + 4.  The payload copy is fused into the checksum pass
 * (Jenkins: one hipMemcpy2DAsync).  out_sums may be NULL. */
int mc_checksum32_encode_batch(int kind, const void *src, size_t src_stride,
                               void *dst, size_t dst_stride, size_t nchunks,
                               size_t chunk_bytes, uint32_t init,
                               const void *prefix, size_t prefix_bytes,
                               int location, uint32_t *out_sums,
                               void *workspace, size_t workspace_bytes,
                               mc_stream_t stream);
/* Checksum32.decode of every encoded row (checksum32.py:64-88): rows of
 * encoded_bytes (payload + 4 checksum bytes at `location`).  Writes the
 * checksum of every payload to out_sums and the stored LE32 value to
 * out_stored (the caller compares them and raises), and, when dst is not
 * NULL, the payloads compacted into dst rows (dst_stride >= encoded_bytes - 4)
 * in the same pass over the encoded bytes (Jenkins: one hipMemcpy2DAsync).
 * Workspace: mc_checksum32_workspace(kind, nchunks, encoded_bytes - 4). */
int mc_checksum32_decode_batch(int kind, const void *src, size_t src_stride,
                               void *dst, size_t dst_stride, size_t nchunks,
                               size_t encoded_bytes, uint32_t init,
                               const void *prefix, size_t prefix_bytes,
                               int location, uint32_t *out_sums,
                               uint32_t *out_stored, void *workspace,
                               size_t workspace_bytes, mc_stream_t stream);

/* Checksum32.encode of ONE chunk (checksum32.py:64-76) in one launch: the
 * payload copy and the checksum in the tiles pass, the last block folds the
 * tile partials and writes the 4 checksum bytes at `location` (and
 * *out_sum if non-NULL).  `ticket` as for mc_fletcher32_verify_fused; NULL
 * (or JenkinsLookup3, whose hash is one serial chain) = the batched entry
 * point with nchunks = 1.  Workspace: mc_checksum32_workspace(kind, 1,
 * chunk_bytes). */
int mc_checksum32_encode_fused(int kind, const void *src, void *dst,
                               size_t chunk_bytes, uint32_t init,
                               const void *prefix, size_t prefix_bytes,
                               int location, uint32_t *out_sum,
                               void *workspace, size_t workspace_bytes,
                               uint32_t *ticket, mc_stream_t stream);
/* Checksum32.decode's verification of ONE encoded buffer (payload + 4 bytes
 * at `location`) in one launch: out_pair[0] = checksum of the payload,
 * out_pair[1] = the stored LE32 value (the caller compares and raises).
 * `ticket`, out_pair and seq as for mc_fletcher32_verify_fused (seq != 0
 * needs a ticket and is refused for Jenkins, which has no one-launch fold);
 * workspace: mc_checksum32_workspace(kind, 1, encoded_bytes - 4), which also
 * covers the aligned path: with location MC_CK_START, a ticket and a 16-B
 * aligned src, CRC32 / CRC32C / Adler32 read the whole buffer with aligned
 * vectors and remove the stored word's share at the finish (same result). */
int mc_checksum32_verify_fused(int kind, const void *src, size_t encoded_bytes,
                               uint32_t init, const void *prefix,
                               size_t prefix_bytes, int location,
                               uint32_t *out_pair, uint32_t seq, void *workspace,
                               size_t workspace_bytes, uint32_t *ticket,
                               mc_stream_t stream);

/* hipStreamSynchronize(stream) (the codecs' one host wait per verified
 * decode); returns a status. */
int mc_stream_synchronize(mc_stream_t stream);
/* The device address of mapped pinned host memory (hipHostGetDevicePointer),
 * NULL if `host` is not mapped: where a kernel may write a host-visible
 * verdict. */
void *mc_host_device_pointer(void *host);
/* A 64-B verdict record {computed, stored, seq, ...} in fine-grained mapped
 * pinned host memory (hipHostMalloc Mapped|Coherent|Portable), seq word 0;
 * NULL on failure.  Pass mc_host_device_pointer(rec) as a fused verify's
 * out_rec/out_pair. */
void *mc_verdict_alloc(void);
void mc_verdict_free(void *rec);
/* Spin until rec[2] == seq (seq != 0), polling hipStreamQuery(stream) every
 * ~1K spins: MC_OK when the record is published; MC_EPROTO if the stream
 * ended without publishing it; the stream's HIP error if it failed.  Replaces
 * the stream synchronisation of a verified decode (~6 us less latency). */
int mc_verdict_wait(const uint32_t *rec, uint32_t seq, mc_stream_t stream);

/* ---- PackBits (packbits.py:33-82) --------------------------------------- */
/* encode n bools (any nonzero byte is True) into dst[0] = padding bits
 * ((8 - n % 8) % 8) followed by np.packbits (MSB first): 1 + ceil(n/8) bytes. */
int mc_packbits(const void *src, void *dst, size_t n, mc_stream_t stream);
/* decode: src = the encoded buffer (header byte first, src_bytes long) into
 * n bools (0/1 bytes); n <= 8 * (src_bytes - 1), normally
 * 8 * (src_bytes - 1) - src[0] (read by the caller). */
int mc_unpackbits(const void *src, size_t src_bytes, void *dst, size_t n,
                  mc_stream_t stream);

/* ---- Blosc shuffle filters (blosc.pyx:67-71, c-blosc shuffle.c) ---------- */
/* Filter a buffer block by block exactly as Blosc does before/after its
 * compressor: the buffer is cut into blocksize-byte blocks (last one
 * shorter); mode MC_BLOSC_SHUFFLE byte-transposes each block's
 * (bsize/typesize, typesize) matrix and copies the bsize % typesize trailing
 * bytes; MC_BLOSC_BITSHUFFLE bit-transposes blocks whose element count is a
 * multiple of 8 (bit k of byte j of element i -> bit i%8 of byte i/8 of
 * plane 8j+k) and copies the others; MC_BLOSC_NOSHUFFLE copies.
 * forward = 1 filters (compress side), 0 inverts (decompress side). */
enum mc_blosc_mode { MC_BLOSC_NOSHUFFLE = 0, MC_BLOSC_SHUFFLE = 1, MC_BLOSC_BITSHUFFLE = 2 };
int mc_blosc_filter(const void *src, void *dst, size_t nbytes, size_t typesize,
                    size_t blocksize, int mode, int forward, mc_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MCODEC_H */
