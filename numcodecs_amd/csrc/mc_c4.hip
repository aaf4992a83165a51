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
//   4 B per element.  A single-pass decoupled look-back variant exists for
//   A/B measurement (MCODEC_C4_VARIANT=2).
// Bit-exact with the reference sequence of codecs (tests/test_gpu_c4.py).
#include <stdlib.h>

#include "mc_scan.h"
#include "mc_shuffle.h"

namespace {

struct C4Params {
  size_t n;      // elements
  McNum off;     // encode: offset in D;   decode: offset in f64
  McNum sc;      // encode: scale in D;    decode: scale in f64
  double rcp;    // decode: RN(1 / scale), computed on the host
  bool fastdiv;  // decode: divide by scale as mul + 2 FMA (mc_div_by_const)
};

template <int D, int A>
MC_DEV int64_t fso_enc(uint64_t xbits, const C4Params &p) {
  McNum v = mc_num_from_bits(xbits, D);
  v = mc_num_binop(v, p.off, MC_OP_SUB, D);
  v = mc_num_binop(v, p.sc, MC_OP_MUL, D);
  v = mc_num_rint(v, D);
  return mc_num_cast(v, D, A).i;
}

template <int D, int A>
MC_DEV uint64_t fso_dec(int64_t a, const C4Params &p) {
  McNum v = mc_num_cast(mc_num_i(a), A, MC_F8);
  if (p.fastdiv) v = mc_num_f(mc_div_by_const(v.f, p.sc.f, p.rcp));
  else v = mc_num_binop(v, p.sc, MC_OP_DIV, MC_F8);
  v = mc_num_binop(v, p.off, MC_OP_ADD, MC_F8);
  return mc_num_to_bits(mc_num_cast(v, MC_F8, D), D);
}

// pack 4 integers of width ES into the quad's ES dwords
template <int ES>
MC_DEV void pack_quad(const int64_t (&d)[4], uint32_t (&w)[ES]) {
  if constexpr (ES == 2) {
    w[0] = ((uint32_t)d[0] & 0xffffu) | ((uint32_t)d[1] << 16);
    w[1] = ((uint32_t)d[2] & 0xffffu) | ((uint32_t)d[3] << 16);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = (uint32_t)d[k];
  }
}

template <int A, int ES>
MC_DEV void unpack_quad(const uint32_t (&w)[ES], int64_t (&d)[4]) {
  if constexpr (ES == 2) {
    d[0] = mc_wrap(w[0] & 0xffffu, A);
    d[1] = mc_wrap(w[0] >> 16, A);
    d[2] = mc_wrap(w[1] & 0xffffu, A);
    d[3] = mc_wrap(w[1] >> 16, A);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = mc_wrap(w[k], A);
  }
}

template <int D, int A, int STEPS = MC_SCAN_STEPS>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_enc(const uint8_t *__restrict__ src,
                                                    uint8_t *__restrict__ dst, C4Params p) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  constexpr int DS = D == MC_F4 ? 4 : 8;
  const size_t tile_e0 = (size_t)blockIdx.x * (4 * STEPS * MC_BLOCK);
  const int lane = threadIdx.x & 63;
  // all steps' loads first (n % 16 == 0: quads are whole)
  uint64_t x[STEPS][4];
#pragma unroll
  for (int q = 0; q < STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    if (e < p.n) {
      mc_load4(src + e * DS, DS, x[q]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) x[q][k] = 0;
    }
  }
#pragma unroll
  for (int q = 0; q < STEPS; ++q) {
    const size_t e = tile_e0 + (size_t)q * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    int64_t a[4], d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = fso_enc<D, A>(x[q][k], p);
    // the element before the quad is the last one of lane - 1's quad; lane 0
    // reads it (A is at most 32 bits wide, so differences mod 2^32 suffice)
    int64_t prev = (int64_t)(int32_t)__shfl_up((uint32_t)a[3], 1, 64);
    if (lane == 0 && e > 0 && e < p.n) prev = fso_enc<D, A>(mc_load_elem(src, e - 1, DS), p);
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

// A thread owns 16 consecutive elements of a 4096-element tile: one 16-B
// (lane-contiguous) load per plane, 4 quads unshuffled in registers.
constexpr int C4_PER = 16;

template <int A, int ES>
MC_DEV void load16_deltas(const uint8_t *src, size_t n, size_t e0, uint32_t (&v)[C4_PER]) {
  mc_u32x4 pl[ES];
#pragma unroll
  for (int b = 0; b < ES; ++b) pl[b] = mc_ld16<true>(src + (size_t)b * n + e0);
#pragma unroll
  for (int c = 0; c < 4; ++c) {  // dword c of every plane = elements 4c..4c+3
    uint32_t pq[ES], w[ES];
#pragma unroll
    for (int b = 0; b < ES; ++b) pq[b] = pl[b][c];
    mc_planes_to_quad<ES>(pq, w);
    int64_t d[4];
    unpack_quad<A, ES>(w, d);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[4 * c + k] = (uint32_t)d[k];
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

// scan of 16 consecutive deltas + FSO decode, staged through LDS for
// lane-contiguous 16-B stores; `pre` = exclusive prefix of the thread.
// The staging image is addressed in 16-B units with unit u stored at
// u ^ ((u >> 3) & 7): a thread's own DS units (written with ds_write_b128,
// 8-lane groups) and the lane-contiguous read-back (ds_read_b128, 16-lane
// groups) are then both conflict-free.  Unswizzled, the 16 ds_write_b32 per
// thread at a 64-B lane stride were 16-way bank conflicts.
MC_DEV int c4_swz(int u) { return u ^ ((u >> 3) & 7); }

template <int D, int A>
MC_DEV void c4_finish(uint8_t *dst, size_t tile, const uint32_t (&incl)[C4_PER], uint32_t pre,
                      uint8_t *outb, const C4Params &p) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  constexpr int UPT = C4_PER * DS / 16;  // 16-B units per thread
  mc_u32x4 *img = reinterpret_cast<mc_u32x4 *>(outb);
  uint32_t o[C4_PER * DS / 4];
#pragma unroll
  for (int k = 0; k < C4_PER; ++k) {
    const uint64_t x = fso_dec<D, A>(mc_wrap((int64_t)(uint32_t)(pre + incl[k]), A), p);
    if constexpr (DS == 4) {
      o[k] = (uint32_t)x;
    } else {
      o[2 * k] = (uint32_t)x;
      o[2 * k + 1] = (uint32_t)(x >> 32);
    }
  }
#pragma unroll
  for (int j = 0; j < UPT; ++j)
    img[c4_swz((int)threadIdx.x * UPT + j)] = mc_u32x4{o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]};
  __syncthreads();
  const size_t tile_b0 = tile * (size_t)MC_SCAN_TILE * DS;
  const size_t nbytes = p.n * DS;
#pragma unroll
  for (int r = 0; r < MC_SCAN_TILE * DS / 16 / MC_BLOCK; ++r) {
    const int u = r * MC_BLOCK + (int)threadIdx.x;
    const size_t off = (size_t)u * 16;
    if (tile_b0 + off < nbytes) mc_st16<true>(dst + tile_b0 + off, img[c4_swz(u)]);
  }
}

template <int D, int A>
MC_DEV void c4_local_scan(const uint8_t *src, size_t tile, const C4Params &p, uint32_t (&v)[C4_PER],
                          uint32_t &run) {
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  if (e0 < p.n) {
    load16_deltas<A, ES>(src, p.n, e0, v);
  } else {
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) v[k] = 0;
  }
  run = 0;
#pragma unroll
  for (int k = 0; k < C4_PER; ++k) {
    run += v[k];
    v[k] = run;
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

// Single-pass decode with decoupled look-back (mc_scan.h): tiles numbered in
// start order, the tile's aggregate published right after its block scan,
// wave 0 walks back 64 predecessors per round.
// COUNTER: tiles numbered by an atomic counter in start order (the counter
// saturates at ~88 increments/us, MI355X_MICROARCH.md "dequeue").  Without
// it the tile is blockIdx.x: with workgroups dispatched in increasing
// blockIdx order per XCD the lowest-numbered waiting tile's predecessors are
// all resident or done, so waits end; if a wait still exceeds the spin bound
// the tile computes its prefix from the data itself, so the result is correct
// under any dispatch order.
template <int D, int A, bool COUNTER>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_decode_lb(const uint8_t *__restrict__ src,
                                                          uint8_t *__restrict__ dst,
                                                          uint32_t *ctrl, uint64_t *status,
                                                          C4Params p, unsigned max_spins) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  __shared__ uint64_t red[MC_BLOCK / 64];
  __shared__ uint32_t slot;
  __shared__ uint32_t prefix_slot;
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * DS];
  __shared__ int ok_slot;
  const size_t tile = COUNTER ? mc_lb_tile(ctrl, &slot) : (size_t)blockIdx.x;
  uint32_t v[C4_PER], run;
  c4_local_scan<D, A>(src, tile, p, v, run);
  uint64_t agg;
  const uint32_t excl = (uint32_t)mc_block_excl_scan<false>(run, red, &agg);
  if (threadIdx.x < 64) {
    bool ok;
    const uint32_t pre = mc_lb_lookback_wave<false>(status, tile, (uint32_t)agg, ok, max_spins);
    if (threadIdx.x == 0) {
      prefix_slot = pre;
      ok_slot = ok;
    }
  }
  __syncthreads();
  if (!ok_slot) {
    // a predecessor never published: sum every delta before this tile from
    // the data itself (correct under any dispatch order), then publish
    constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
    uint32_t acc = 0;
    for (size_t e = (size_t)threadIdx.x * C4_PER; e < tile * MC_SCAN_TILE; e += MC_BLOCK * C4_PER) {
      uint32_t w[C4_PER];
      load16_deltas<A, ES>(src, p.n, e, w);
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) acc += w[k];
    }
    uint64_t tot;
    mc_block_excl_scan<false>(acc, red, &tot);
    if (threadIdx.x == 0) {
      prefix_slot = (uint32_t)tot;
      mc_lb_publish_inclusive(status, tile, (uint32_t)tot + (uint32_t)agg);
    }
    __syncthreads();
  }
  c4_finish<D, A>(dst, tile, v, prefix_slot + excl, outb, p);
}

// Single-pass decode over coarse partitions (variants 5/6): a workgroup holds
// R consecutive 4096-element tiles in registers (one pass over the data),
// scans them locally (one block scan of R values at once), publishes the
// partition's aggregate and walks back 256 predecessors per round
// (mc_lb_lookback_wave4): R times fewer hand-offs than one per tile.
template <int R>
MC_DEV void c4_block_excl_scan_multi(const uint32_t (&x)[R], uint32_t (&excl)[R], uint32_t (&tot)[R],
                                     uint32_t (*red)[MC_BLOCK / 64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    incl[r] = x[r];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(incl[r], off, 64);
      if (lane >= off) incl[r] += o;
    }
  }
  if (lane == 63) {
#pragma unroll
    for (int r = 0; r < R; ++r) red[r][wave] = incl[r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    uint32_t wpre = 0, t = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) {
      const uint32_t val = red[r][w];
      if (w < wave) wpre += val;
      t += val;
    }
    excl[r] = wpre + incl[r] - x[r];
    tot[r] = t;
  }
  __syncthreads();
}

template <int D, int A, int R>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_decode_lbp(const uint8_t *__restrict__ src,
                                                           uint8_t *__restrict__ dst,
                                                           uint64_t *status, C4Params p,
                                                           unsigned max_spins) {
  constexpr int DS = D == MC_F4 ? 4 : 8;
  constexpr int ES = A == MC_I2 || A == MC_U2 ? 2 : 4;
  __shared__ uint32_t red[R][MC_BLOCK / 64];
  __shared__ uint64_t red1[MC_BLOCK / 64];
  __shared__ uint32_t prefix_slot;
  __shared__ int ok_slot;
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * DS];
  const size_t part = blockIdx.x;
  const size_t tile0 = part * R;
  uint32_t v[R][C4_PER];
#pragma unroll
  for (int r = 0; r < R; ++r) {  // every load of the partition first
    const size_t e0 = (tile0 + r) * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
    if (e0 < p.n) {
      load16_deltas<A, ES>(src, p.n, e0, v[r]);
    } else {
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) v[r][k] = 0;
    }
  }
  uint32_t run[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    run[r] = 0;
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) {
      run[r] += v[r][k];
      v[r][k] = run[r];
    }
  }
  uint32_t excl[R], tot[R];
  c4_block_excl_scan_multi<R>(run, excl, tot, red);
  uint32_t agg = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) agg += tot[r];
  if (threadIdx.x < 64) {
    bool ok;
    const uint32_t pre = mc_lb_lookback_wave4<false>(status, part, agg, ok, max_spins);
    if (threadIdx.x == 0) {
      prefix_slot = pre;
      ok_slot = ok;
    }
  }
  __syncthreads();
  if (!ok_slot) {  // a predecessor never published: derive the prefix from the data
    uint32_t acc = 0;
    for (size_t e = (size_t)threadIdx.x * C4_PER; e < tile0 * MC_SCAN_TILE; e += MC_BLOCK * C4_PER) {
      uint32_t w[C4_PER];
      load16_deltas<A, ES>(src, p.n, e, w);
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) acc += w[k];
    }
    uint64_t t;
    mc_block_excl_scan<false>(acc, red1, &t);
    if (threadIdx.x == 0) {
      prefix_slot = (uint32_t)t;
      mc_lb_publish_inclusive(status, part, (uint32_t)t + agg);
    }
    __syncthreads();
  }
  uint32_t base = prefix_slot;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if ((tile0 + r) * MC_SCAN_TILE < p.n) c4_finish<D, A>(dst, tile0 + r, v[r], base + excl[r], outb, p);
    base += tot[r];
    __syncthreads();  // outb is reused by the next tile
  }
}

template <int D, int A>
static void c4_decode_lbp(const uint8_t *s, uint8_t *d, uint8_t *ws, const C4Params &p, int R,
                          unsigned max_spins, hipStream_t st) {
  const size_t ntiles = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  uint64_t *status = reinterpret_cast<uint64_t *>(ws + 16);
  if (R == 8) {
    const unsigned g = (unsigned)((ntiles + 7) / 8);
    k_c4_decode_lbp<D, A, 8><<<g, MC_BLOCK, 0, st>>>(s, d, status, p, max_spins);
  } else {
    const unsigned g = (unsigned)((ntiles + 3) / 4);
    k_c4_decode_lbp<D, A, 4><<<g, MC_BLOCK, 0, st>>>(s, d, status, p, max_spins);
  }
}

// the workspace (tile counter + status words) is zeroed by the caller
template <int D, int A>
static void c4_decode_lb(const uint8_t *s, uint8_t *d, uint8_t *ws, const C4Params &p, bool counter,
                         unsigned max_spins, hipStream_t st) {
  const size_t ntiles = (p.n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  if (counter)
    k_c4_decode_lb<D, A, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(
        s, d, reinterpret_cast<uint32_t *>(ws), reinterpret_cast<uint64_t *>(ws + 16), p, max_spins);
  else
    k_c4_decode_lb<D, A, false><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(
        s, d, reinterpret_cast<uint32_t *>(ws), reinterpret_cast<uint64_t *>(ws + 16), p, max_spins);
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

// MCODEC_C4_VARIANT: 2 = single-pass look-back decode with an atomic tile
// counter, 3 = look-back in blockIdx order, 4 = blockIdx order with the
// data-derived fallback forced (tests); the default is chosen in DESIGN.md
// decode variant used when neither the caller nor MCODEC_C4_VARIANT picks
// one: 1 = three-pass scan (DESIGN.md records the A/B that chose it)
constexpr int C4_DEFAULT_VARIANT = 1;

static int mc_c4_variant() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("MCODEC_C4_VARIANT");
    v = e ? atoi(e) : 0;
  }
  return v;
}

static bool c4_ok(const void *src, const void *dst, size_t n, int dtype, int astype) {
  if (!(dtype == MC_F4 || dtype == MC_F8)) return false;
  if (!(astype == MC_I2 || astype == MC_U2 || astype == MC_I4 || astype == MC_U4)) return false;
  if (n % 16 != 0) return false;  // 16-B plane accesses (decode)
  return src && dst && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0;
}

#define MC_C4_DISPATCH(FN, ...)                                              \
  do {                                                                       \
    if (dtype == MC_F4) {                                                    \
      switch (astype) {                                                      \
        case MC_I2: FN<MC_F4, MC_I2>(__VA_ARGS__); break;                    \
        case MC_U2: FN<MC_F4, MC_U2>(__VA_ARGS__); break;                    \
        case MC_I4: FN<MC_F4, MC_I4>(__VA_ARGS__); break;                    \
        default: FN<MC_F4, MC_U4>(__VA_ARGS__); break;                       \
      }                                                                      \
    } else {                                                                 \
      switch (astype) {                                                      \
        case MC_I2: FN<MC_F8, MC_I2>(__VA_ARGS__); break;                    \
        case MC_U2: FN<MC_F8, MC_U2>(__VA_ARGS__); break;                    \
        case MC_I4: FN<MC_F8, MC_I4>(__VA_ARGS__); break;                    \
        default: FN<MC_F8, MC_U4>(__VA_ARGS__); break;                       \
      }                                                                      \
    }                                                                        \
  } while (0)

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

size_t mc_fso_delta_shuffle_decode_workspace(size_t n) {
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t scan3 = 24 * ((ntiles + 1) / 2);  // pair totals, first values, pair prefixes
  return mc_lb_workspace(ntiles) > scan3 ? mc_lb_workspace(ntiles) : scan3;
}

int mc_fso_delta_shuffle_decode_variant(const void *src, void *dst, size_t n, int astype, int dtype,
                                        double scale, double offset, void *workspace,
                                        size_t workspace_bytes, int variant, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, dtype, astype)) return MC_EINVAL;
  if (variant < 0 || variant > 7) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_fso_delta_shuffle_decode_workspace(n)) return MC_ENOSPC;
  C4Params p;
  p.n = n;
  p.off = mc_num_f(offset);
  p.sc = mc_num_f(scale);
  p.rcp = 1.0 / scale;
  p.fastdiv = mc_fastdiv_ok(scale);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  if (variant == 0) variant = mc_c4_variant() ? mc_c4_variant() : C4_DEFAULT_VARIANT;
  if (n % 16 == 0 && variant >= 5) {  // coarse partitions: 5 = 4 tiles, 6 = 8 tiles, 7 = 4 forced fallback
    uint8_t *ws = static_cast<uint8_t *>(workspace);
    const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
    const int rc = mc_hip_status(hipMemsetAsync(ws, 0, mc_lb_workspace(ntiles), st));
    if (rc != MC_OK) return rc;
    const unsigned spins = variant == 7 ? 0u : MC_LB_WAVE_SPINS;
    const int R = variant == 6 ? 8 : 4;
    MC_C4_DISPATCH(c4_decode_lbp, s, d, ws, p, R, spins, st);
  } else if (n % 16 == 0 && (variant == 2 || variant == 3 || variant == 4)) {
    uint8_t *ws = static_cast<uint8_t *>(workspace);
    const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
    const int rc = mc_hip_status(hipMemsetAsync(ws, 0, mc_lb_workspace(ntiles), st));
    if (rc != MC_OK) return rc;
    const bool counter = variant == 2;
    // variant 4 (tests): no waiting at all, every tile whose predecessor has
    // not published yet takes the data-derived fallback
    const unsigned spins = variant == 4 ? 0u : MC_LB_WAVE_SPINS;
    MC_C4_DISPATCH(c4_decode_lb, s, d, ws, p, counter, spins, st);
  } else {
    uint64_t *sums = static_cast<uint64_t *>(workspace);
    MC_C4_DISPATCH(c4_decode, s, d, sums, p, st);
  }
  return mc_last_launch();
}

int mc_fso_delta_shuffle_decode(const void *src, void *dst, size_t n, int astype, int dtype,
                                double scale, double offset, void *workspace,
                                size_t workspace_bytes, mc_stream_t stream) {
  return mc_fso_delta_shuffle_decode_variant(src, dst, n, astype, dtype, scale, offset, workspace,
                                             workspace_bytes, 0, stream);
}

}  // extern "C"
