// mc_c4.hip -- fused FixedScaleOffset -> Delta -> Shuffle chunk pipeline
// (BASELINE configs[3]: FSO(offset, scale, f4 -> i2) -> Delta(i2) ->
// Shuffle(2)), the composition of fixedscaleoffset.py:83-113, delta.py:52-83
// and _shuffle.pyx:11-30 that a Zarr array with filters
// [FixedScaleOffset, Delta] and a shuffle applies per chunk.
//
// encode, one pass: each lane loads 4 consecutive float elements (and the
//   element before them), applies FSO encode exactly as numpy does it in the
//   float dtype (NEP 50: Python scalars are weak), takes wrap-around
//   differences in the integer dtype, and writes the 4 integers as plane
//   dwords of the shuffled chunk (4x4 byte transpose in registers).
//   HBM: read 4 (or 8) B + write 2 (or 4) B per element.
// decode, three passes over 4096-element tiles (mc_scan.h), each thread
//   owning 16 consecutive elements: per-tile totals of the unshuffled deltas;
//   exclusive scan of the totals (one workgroup); rescan of each tile + FSO
//   decode ((x / scale + offset) in float64, then cast to the float dtype),
//   staged through LDS for coalesced stores.  HBM: read 2 B twice + write
//   4 B per element.  (Single-pass decoupled look-back schedules were
//   measured slower and live in tools/lab/lab_c4.hip, outside this library.)
// Bit-exact with the reference sequence of codecs (tests/test_gpu_c4.py).
#include "mc_c4.h"

namespace {

// blockIdx.y = chunk of a batch (row r at src + r * src_stride, dst + r *
// dst_stride; one chunk: y = 0, strides unused)
template <int D, int A, int STEPS = MC_SCAN_STEPS>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_enc(const uint8_t *__restrict__ src,
                                                    uint8_t *__restrict__ dst, C4Params p,
                                                    size_t src_stride = 0, size_t dst_stride = 0) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  constexpr int DS = D == MC_F4 ? 4 : 8;
  src += (size_t)blockIdx.y * src_stride;
  dst += (size_t)blockIdx.y * dst_stride;
  const size_t tile_e0 = (size_t)blockIdx.x * (4 * STEPS * MC_BLOCK);
  const int lane = threadIdx.x & 63;
  // all steps' loads first (n % 16 == 0: quads are whole), with lane 0's
  // element before its quad (the last of the previous wave's quads, read
  // from memory) -- loaded in the second loop, each was waited for on its
  // own: STEPS extra round trips per workgroup (round 5)
  uint64_t x[STEPS][4], before[STEPS];
#pragma unroll
  for (int q = 0; q < STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    if (e < p.n) {
      mc_load4(src + e * DS, DS, x[q]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) x[q][k] = 0;
    }
    before[q] = lane == 0 && e > 0 && e < p.n ? mc_load_elem(src, e - 1, DS) : 0;
  }
#pragma unroll
  for (int q = 0; q < STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    int64_t a[4], d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = fso_enc<D, A>(x[q][k], p);
    // the element before the quad is the last one of lane - 1's quad; lane 0
    // reads it (A is at most 32 bits wide, so differences mod 2^32 suffice)
    int64_t prev = (int64_t)(int32_t)mc_wave_shr1((uint32_t)a[3], 0u);
    if (lane == 0 && e > 0 && e < p.n) prev = fso_enc<D, A>(before[q], p);
    if (e >= p.n) continue;
    d[0] = e > 0 ? mc_wrap(a[0] - prev, A) : a[0];
#pragma unroll
    for (int k = 1; k < 4; ++k) d[k] = mc_wrap(a[k] - a[k - 1], A);
    uint32_t w[ES], pl[ES];
    pack_quad<ES>(d, w);
    mc_quad_to_planes<ES>(w, pl);
#pragma unroll
    for (int b = 0; b < ES; ++b) mc_st4<true>(dst + (size_t)b * p.n + e, pl[b]);
  }
}

// Reduce pass over PAIRS of 4096-element tiles (one workgroup, four 16-B
// loads per thread in flight): pair_sums[i] = total of tiles 2i and 2i+1,
// first[i] = total of tile 2i.  The scan then runs over half as many values
// (k_scan_sums: 8K totals in one round instead of 16K in two), and the apply
// pass takes tile t's prefix as scan[t/2] + (t odd ? first[t/2] : 0).
template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_reduce2(const uint8_t *__restrict__ src,
                                                        uint64_t *__restrict__ pair_sums,
                                                        uint64_t *__restrict__ first, C4Params p) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  __shared__ uint64_t lds[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t e0 = (size_t)blockIdx.x * 2 * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  uint32_t acc[2] = {0, 0};
  uint32_t v[2][C4_PER];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (e0 + h * MC_SCAN_TILE < p.n) load16_deltas<A, ES>(src, p.n, e0 + h * MC_SCAN_TILE, v[h]);
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (e0 + h * MC_SCAN_TILE < p.n) {
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) acc[h] += v[h][k];
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc[0] += __shfl_xor(acc[0], off, 64);
    acc[1] += __shfl_xor(acc[1], off, 64);
  }
  if (lane == 0) {
    lds[0][wave] = acc[0];
    lds[1][wave] = acc[1];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0, b = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) {
      a += (uint32_t)lds[0][w];
      b += (uint32_t)lds[1][w];
    }
    first[blockIdx.x] = a;
    pair_sums[blockIdx.x] = (uint32_t)(a + b);
  }
}

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_apply(const uint8_t *__restrict__ src,
                                                      uint8_t *__restrict__ dst,
                                                      const uint64_t *__restrict__ pair_pre,
                                                      const uint64_t *__restrict__ first,
                                                      C4Params p) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  __shared__ uint32_t red[MC_BLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * DS];
  const size_t tile = blockIdx.x;
  uint32_t v[C4_PER], run;
  c4_local_scan<D, A>(src, tile, p, v, run);
  uint32_t agg;
  const uint32_t excl = mc_block_excl_scan32(run, red, &agg);
  const uint32_t tile_pre = (uint32_t)pair_pre[tile >> 1] + ((tile & 1) ? (uint32_t)first[tile >> 1] : 0u);
  c4_finish<D, A>(dst, tile, v, tile_pre + excl, outb, p);
}

// Batched decode (Zarr chunk pipelines): one workgroup per chunk walks its
// tiles with a running carry -- a single pass, the next tile's planes in
// flight while the current one is scanned and stored; thousands of chunks
// fill the chip.  Same per-tile code as k_c4_apply.
// Few large chunks would leave the chip under-filled with one workgroup per
// chunk, so a chunk may be cut into `nseg` segments of whole tiles (grid =
// chunks x segments): segment s starts from the sum of the earlier
// segments' totals (seg_tot[c * nseg + s'], k_c4_seg_reduce) -- one extra
// read of the encoded planes, in exchange for enough workgroups.
template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_seg_reduce(const uint8_t *__restrict__ src, size_t src_stride,
                                                           uint32_t *__restrict__ seg_tot, unsigned nseg, C4Params p) {
  constexpr int ES = c4_es<A>();
  __shared__ uint32_t red[MC_BLOCK / 64];
  const size_t c = blockIdx.x / nseg;
  const unsigned sg = blockIdx.x - (unsigned)(c * nseg);
  src += c * src_stride;
  const size_t ntiles = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t t0 = ntiles * sg / nseg, t1 = ntiles * (sg + 1) / nseg;
  uint32_t acc = 0;
  for (size_t t = t0; t < t1; t += 2) {  // two tiles' planes in flight
    uint32_t v[2][C4_PER];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const size_t e0 = (t + h) * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
      if (t + h < t1 && e0 < p.n) {
        load16_deltas<A, ES, false>(src, p.n, e0, v[h]);  // default policy: re-read by the decode pass
      } else {
#pragma unroll
        for (int k = 0; k < C4_PER; ++k) v[h][k] = 0;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) acc += v[h][k];
  }
  uint32_t tot;
  (void)mc_block_excl_scan32(acc, red, &tot);
  if (threadIdx.x == 0) seg_tot[blockIdx.x] = tot;
}

template <int D, int A, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_dec_rows(const uint8_t *__restrict__ src, size_t src_stride,
                                                         uint8_t *__restrict__ dst, size_t dst_stride, C4Params p,
                                                         const uint32_t *__restrict__ seg_tot = nullptr,
                                                         unsigned nseg = 1) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  constexpr int ES = c4_es<A>();
  __shared__ uint32_t red[MC_BLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * DS];
  const size_t c = blockIdx.x / nseg;
  const unsigned sg = blockIdx.x - (unsigned)(c * nseg);
  src += c * src_stride;
  dst += c * dst_stride;
  const size_t ntiles_all = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t tfirst = ntiles_all * sg / nseg, ntiles = ntiles_all * (sg + 1) / nseg;
  uint32_t nxt[C4_PER];
  auto load = [&](size_t tile, uint32_t (&v)[C4_PER]) {
    const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
    if (e0 < p.n) {
      load16_deltas<A, ES, NT>(src, p.n, e0, v);
    } else {
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) v[k] = 0;
    }
  };
  if (tfirst >= ntiles) return;
  load(tfirst, nxt);
  uint32_t carry = 0;
  if (sg) {  // the earlier segments' totals, summed by the whole block
    uint32_t x = 0;
    for (unsigned j = threadIdx.x; j < sg; j += MC_BLOCK) x += seg_tot[c * nseg + j];
    (void)mc_block_excl_scan32(x, red, &carry);
  }
  for (size_t t = tfirst; t < ntiles; ++t) {
    uint32_t v[C4_PER];
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) v[k] = nxt[k];
    if (t + 1 < ntiles) load(t + 1, nxt);
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) {
      run += v[k];
      v[k] = run;
    }
    uint32_t tot;
    const uint32_t excl = mc_block_excl_scan32(run, red, &tot);
    c4_finish<D, A>(dst, t, v, carry + excl, outb, p);
    carry += tot;
  }
}

template <int D, int A>
static void c4_encode_batch(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t nchunks, const C4Params &p,
                            hipStream_t st) {
  const unsigned tiles = (unsigned)((p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE);
  for (size_t c0 = 0; c0 < nchunks; c0 += 65535) {
    const unsigned rows = (unsigned)(nchunks - c0 < 65535 ? nchunks - c0 : 65535);
    k_c4_enc<D, A><<<dim3(tiles, rows), MC_BLOCK, 0, st>>>(s + c0 * ss, d + c0 * ds, p, ss, ds);
  }
}

// segments per chunk: enough workgroups to fill the chip (>= 2048), whole
// tiles, none when the batch alone fills it
static unsigned c4_batch_segments(size_t nchunks, size_t n) {
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  size_t seg = nchunks >= 2048 ? 1 : (2048 + nchunks - 1) / nchunks;
  if (seg > ntiles) seg = ntiles;
  if (seg > 4096) seg = 4096;
  return (unsigned)(seg ? seg : 1);
}

// Segmented decodes run in groups of rows whose encoded planes the second
// pass re-reads partly from the Infinity Cache (256 MiB MALL).  Measured on
// 256 x 4 MiB / 16 x 64 MiB f4<-i2 (tools/probe_c4_batch.py): one group 414 /
// 425 us; groups of 16 Mi elements 434 / 480 (more launch pairs); 64 Mi 364 /
// 383; 128 Mi 360 / 363 (357 / 364 split evenly); 96 Mi and 192 Mi, with a
// short last group, 403-450.  Default 128 Mi elements, split evenly
// (mc_sched.c4_group_mi; the lab overrides it).
struct C4Plan {
  size_t rows;    // chunks per group (launch pair)
  unsigned nseg;  // segments per chunk
};

static size_t c4_group_elems() {
  const int v = mc_sched.c4_group_mi;  // mc_sched.h
  return (size_t)(v > 0 ? v : 128) << 20;
}

static C4Plan c4_batch_plan(size_t nchunks, size_t n) {
  if (c4_batch_segments(nchunks, n) == 1) return {nchunks, 1};
  size_t g = c4_group_elems() / n;
  if (g < 1) g = 1;
  if (g > nchunks) g = nchunks;
  const size_t ngroups = (nchunks + g - 1) / g;
  g = (nchunks + ngroups - 1) / ngroups;  // even groups: a short last group costs a whole launch pair
  const unsigned nseg = c4_batch_segments(g, n);
  return nseg > 1 ? C4Plan{g, nseg} : C4Plan{nchunks, 1};
}

template <int D, int A>
static void c4_decode_batch(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t nchunks, const C4Params &p,
                            uint32_t *seg_tot, hipStream_t st) {
  const C4Plan plan = c4_batch_plan(nchunks, p.n);
  const unsigned nseg = plan.nseg;
  const size_t per_launch = nseg > 1 ? plan.rows : ((size_t)1 << 30);
  for (size_t c0 = 0; c0 < nchunks; c0 += per_launch) {
    const size_t rows = nchunks - c0 < per_launch ? nchunks - c0 : per_launch;
    const unsigned grid = (unsigned)(rows * nseg);
    if (nseg > 1) {  // segments: the second pass re-reads what the first read (default-policy loads)
      k_c4_seg_reduce<D, A><<<grid, MC_BLOCK, 0, st>>>(s + c0 * ss, ss, seg_tot, nseg, p);
      k_c4_dec_rows<D, A, false><<<grid, MC_BLOCK, 0, st>>>(s + c0 * ss, ss, d + c0 * ds, ds, p, seg_tot, nseg);
    } else {
      k_c4_dec_rows<D, A, true><<<grid, MC_BLOCK, 0, st>>>(s + c0 * ss, ss, d + c0 * ds, ds, p, seg_tot, nseg);
    }
  }
}

template <int D, int A>
static void c4_encode(const uint8_t *s, uint8_t *d, const C4Params &p, hipStream_t st) {
  // 4 quads per thread: 8 and 16 measured slower (77.6 / 93.0 vs 70.6 us for
  // n = 64 Mi, register pressure)
  const unsigned grid = (unsigned)((p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE);
  k_c4_enc<D, A><<<grid, MC_BLOCK, 0, st>>>(s, d, p);
}

template <int D, int A>
static void c4_decode(const uint8_t *s, uint8_t *d, uint64_t *sums, const C4Params &p,
                      hipStream_t st) {
  const size_t ntiles = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t npairs = (ntiles + 1) / 2;  // workspace: 3 * 8 * npairs bytes
  uint64_t *pair = sums, *first = sums + npairs, *pre = sums + 2 * npairs;
  k_c4_reduce2<D, A><<<(unsigned)npairs, MC_BLOCK, 0, st>>>(s, pair, first, p);
  mc_launch_scan_sums_mw<false>(pair, pre, npairs, st);
  k_c4_apply<D, A><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, pre, first, p);
}

// ---------------------------------------------------------------------------
// Two-launch decode (the default when the caller passes an arrival `ticket`):
// the scan of the tile totals is folded into the two passes, and the apply
// pass's re-read of the encoded planes is partly served by the 256 MiB
// Infinity Cache.
//  * k_c4_reduce_g: a workgroup covers a PAIR of tiles (four 16-B loads per
//    thread in flight, default-policy loads: the lines stay in the Infinity
//    Cache for the apply pass), stores the two tile totals and adds the
//    pair's total into its GROUP's word (GT tiles per group, at most 64
//    groups) with ONE returning 64-bit atomic: word = (sum << 16) + count on
//    the group's own 128-B line of `ticket` (the count never carries into the
//    sum; sums are needed mod 2^32).  The group's last arriver writes
//    gtot[g] and zeroes the word, so the ticket is left zero.
//  * k_c4_apply_g: prefix of tile t = sum(gtot[0..g)) + the totals of the
//    tiles of group g before t -- both loaded before the tile's data and
//    folded into the block scan's one LDS round.
// Measured on MI355X for n = 64 Mi (tools/probe_c4_2l.py, lab_mall.hip):
// 95-99 us for the 3-pass scan (reduce 22, sums 6, apply 66) against
// 83-86 us (reduce 25, apply 58: the temporal loads make about half the
// re-read an Infinity-Cache hit; slabs that would make all of it one cost
// more in launches than they saved).
// ---------------------------------------------------------------------------
constexpr unsigned C4_MAX_GROUPS = 64;

static inline unsigned c4_group_tiles(size_t ntiles) {
  unsigned gt = 256;  // tiles per group: at most 64 groups
  while ((ntiles + gt - 1) / gt > C4_MAX_GROUPS) gt *= 2;
  return gt;
}

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_reduce_g(const uint8_t *__restrict__ src, uint32_t *ws,
                                                         uint32_t *ticket, C4Params p, size_t ntiles, unsigned GT) {
  constexpr int ES = c4_es<A>();
  __shared__ uint32_t lds[2][MC_BLOCK / 64];
  uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t t0 = (size_t)blockIdx.x * 2;
  const size_t e0 = t0 * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  uint32_t acc[2] = {0, 0};
  uint32_t v[2][C4_PER];
  if ((t0 + 2) * MC_SCAN_TILE <= p.n) {
    // both tiles in range: the loads unbranched, all in flight together
    // (bounds-branched, the second tile's waited for the first's, round 5)
#pragma unroll
    for (int h = 0; h < 2; ++h) load16_deltas<A, ES, false>(src, p.n, e0 + h * MC_SCAN_TILE, v[h]);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) acc[h] += v[h][k];
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (e0 + h * MC_SCAN_TILE < p.n) load16_deltas<A, ES, false>(src, p.n, e0 + h * MC_SCAN_TILE, v[h]);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (e0 + h * MC_SCAN_TILE < p.n) {
#pragma unroll
        for (int k = 0; k < C4_PER; ++k) acc[h] += v[h][k];
      }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc[0] += __shfl_xor(acc[0], off, 64);
    acc[1] += __shfl_xor(acc[1], off, 64);
  }
  if (lane == 0) {
    lds[0][wave] = acc[0];
    lds[1][wave] = acc[1];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t tot = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t a = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) a += lds[h][w];
    if (t0 + h < ntiles) tile_tot[t0 + h] = a;
    tot += a;
  }
  const size_t g = t0 / GT;
  const size_t in_group = ntiles - g * GT < GT ? ntiles - g * GT : GT;
  const unsigned long long arrivals = (in_group + 1) / 2;  // workgroups (pairs) of group g
  unsigned long long *word = reinterpret_cast<unsigned long long *>(ticket + (size_t)MC_ARRIVAL_LINE * g);
  const unsigned long long old = atomicAdd(word, ((unsigned long long)tot << 16) | 1ull);
  if ((old & 0xffffu) + 1u == arrivals) {
    gtot[g] = (uint32_t)(old >> 16) + tot;
    *word = 0;  // every arrival of this call is in: left zero
  }
}

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_apply_g(const uint8_t *__restrict__ src,
                                                        uint8_t *__restrict__ dst, const uint32_t *ws, C4Params p,
                                                        size_t ntiles, unsigned GT) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  constexpr int ES = c4_es<A>();
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * DS];
  const uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const size_t tile = blockIdx.x;
  const size_t g = tile / GT, gt0 = g * GT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the data loads first, then the prefix pieces, all in flight together
  // (k_dscan_apply_g: a loop-carried prefix sum between them made every
  // workgroup wait for the prefix words before its data loads issued)
  uint32_t v[C4_PER];
  const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  const bool in = e0 < p.n;
  mc_u32x4 pl[ES];
  if (in) {  // raw plane vectors only: converted after the prefix loads issued
#pragma unroll
    for (int b = 0; b < ES; ++b) pl[b] = mc_ld16<false>(src + (size_t)b * p.n + e0);
  }
  const uint32_t xg = (wave == 0 && (size_t)lane < g) ? gtot[lane] : 0u;
  auto tile_tots = [&](unsigned j0) {  // 8 of the group's earlier tile totals per thread
    uint32_t tt[8], y = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t j = j0 + (size_t)u * MC_BLOCK + threadIdx.x;
      tt[u] = (j < GT && gt0 + j < tile) ? tile_tot[gt0 + j] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) y += tt[u];
    return y;
  };
  uint32_t x = tile_tots(0);
  for (unsigned j0 = 8 * MC_BLOCK; j0 < GT; j0 += 8 * MC_BLOCK) x += tile_tots(j0);
  x += xg;
  if (in) {
    c4_planes_to_deltas<A, ES>(pl, v);
  } else {
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) v[k] = 0;
  }
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < C4_PER; ++k) {
    run += v[k];
    v[k] = run;
  }
  // one LDS round: the exclusive scan of `run` and the block sum of `x`
  uint32_t incl = run;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  if (lane == 63) red[0][wave] = incl;
  if (lane == 0) red[1][wave] = x;
  __syncthreads();
  uint32_t pre = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) {
    if (w < wave) pre += red[0][w];
    pre += red[1][w];
  }
  c4_finish<D, A>(dst, tile, v, pre + (incl - run), outb, p);
}

template <int D, int A>
static void c4_decode_g(const uint8_t *s, uint8_t *d, uint32_t *ws, uint32_t *ticket, const C4Params &p,
                        hipStream_t st) {
  const size_t ntiles = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const unsigned gt = c4_group_tiles(ntiles);
  k_c4_reduce_g<D, A><<<(unsigned)((ntiles + 1) / 2), MC_BLOCK, 0, st>>>(s, ws, ticket, p, ntiles, gt);
  k_c4_apply_g<D, A><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, ws, p, ntiles, gt);
}

}  // namespace

extern "C" {

int mc_fso_delta_shuffle_encode(const void *src, void *dst, size_t n, int dtype, int astype,
                                double offset, double scale, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, dtype, astype)) return MC_EINVAL;
  C4Params p;
  p.n = n;
  p.off = mc_num_f(offset);
  p.sc = mc_num_f(scale);
  p.rcp = 0.0;
  p.fastdiv = false;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  MC_C4_DISPATCH(c4_encode, s, d, p, st);
  return mc_last_launch();
}

static bool c4_batch_ok(const void *src, size_t ss, const void *dst, size_t ds, size_t nchunks, size_t n, int dtype,
                        int astype) {
  if (!c4_ok(src, dst, n, dtype, astype)) return false;
  if (nchunks > 1 && (ss % 16 || ds % 16 || ss < n * (size_t)mc_itemsize(dtype) ||
                      ds < n * (size_t)mc_itemsize(astype)))
    return false;
  return true;
}

int mc_fso_delta_shuffle_encode_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                                      size_t nchunks, size_t n, int dtype, int astype, double offset, double scale,
                                      mc_stream_t stream) {
  if (n == 0 || nchunks == 0) return MC_OK;
  if (!c4_batch_ok(src, src_stride, dst, dst_stride, nchunks, n, dtype, astype)) return MC_EINVAL;
  C4Params p;
  p.n = n;
  p.off = mc_num_f(offset);
  p.sc = mc_num_f(scale);
  p.rcp = 0.0;
  p.fastdiv = false;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  MC_C4_DISPATCH(c4_encode_batch, s, src_stride, d, dst_stride, nchunks, p, st);
  return mc_last_launch();
}

size_t mc_fso_delta_shuffle_decode_batch_workspace(size_t nchunks, size_t n) {
  const C4Plan plan = c4_batch_plan(nchunks, n);
  return plan.nseg > 1 ? plan.rows * plan.nseg * sizeof(uint32_t) : 0;
}

int mc_fso_delta_shuffle_decode_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                                      size_t nchunks, size_t n, int astype, int dtype, double scale, double offset,
                                      void *workspace, size_t workspace_bytes, mc_stream_t stream) {
  if (n == 0 || nchunks == 0) return MC_OK;
  if (!c4_batch_ok(dst, dst_stride, src, src_stride, nchunks, n, dtype, astype)) return MC_EINVAL;
  const size_t need = mc_fso_delta_shuffle_decode_batch_workspace(nchunks, n);
  if (need && (!workspace || workspace_bytes < need || (uintptr_t)workspace % 4)) return MC_ENOSPC;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint32_t *seg = static_cast<uint32_t *>(workspace);
  hipStream_t st = (hipStream_t)stream;
  MC_C4_DISPATCH(c4_decode_batch, s, src_stride, d, dst_stride, nchunks, p, seg, st);
  return mc_last_launch();
}

size_t mc_fso_delta_shuffle_decode_workspace(size_t n) {
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t three_pass = 24 * ((ntiles + 1) / 2);  // pair totals, first values, pair prefixes
  const size_t two_launch = 4 * (ntiles + C4_MAX_GROUPS);  // tile totals, group totals
  return three_pass > two_launch ? three_pass : two_launch;
}

int mc_fso_delta_shuffle_decode(const void *src, void *dst, size_t n, int astype, int dtype,
                                double scale, double offset, void *workspace,
                                size_t workspace_bytes, uint32_t *ticket, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, dtype, astype)) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_fso_delta_shuffle_decode_workspace(n)) return MC_ENOSPC;
  if (ticket && (uintptr_t)ticket % 8) return MC_EINVAL;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  // the two-launch decode needs a ticket and groups of at most 1024 tiles
  // (the apply workgroup sums its group's earlier tile totals, 4 per thread)
  if (ticket && c4_group_tiles(ntiles) <= 1024) {
    uint32_t *ws = static_cast<uint32_t *>(workspace);
    MC_C4_DISPATCH(c4_decode_g, s, d, ws, ticket, p, st);
  } else {
    uint64_t *sums = static_cast<uint64_t *>(workspace);
    MC_C4_DISPATCH(c4_decode, s, d, sums, p, st);
  }
  return mc_last_launch();
}

}  // extern "C"
