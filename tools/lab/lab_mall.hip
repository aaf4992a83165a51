// lab_mall.hip -- LAB ONLY (libmcodec_lab.so).  Does the three-pass C4
// decode's second read of the encoded planes come from the 256 MB Infinity
// Cache (MALL) when the two passes walk the chunk in OPPOSITE orders?
//
// The product's reduce and apply passes both walk tiles in increasing order,
// so the apply pass re-reads tile t after the reduce pass has read every
// other tile and the apply pass has moved 3x as much again: a reuse distance
// larger than the MALL for most of the chunk.  With the reduce pass walking
// the tiles from the END (blockIdx -> last tile first; workgroups are
// dispatched in blockIdx order), the tiles the apply pass needs first are the
// ones the reduce pass read last.  flags:
//   bit 0  reduce pass in reverse tile order
//   bit 1  reduce pass with default-policy (temporal) loads instead of nt
//   bit 2  apply pass with default-policy loads
//   bit 3  apply pass in reverse tile order
// FixedScaleOffset(f4 <- i2) <- Delta(i2) <- Shuffle(2) only (the BASELINE C4
// config); identical bytes to mc_fso_delta_shuffle_decode for every flag.
#include "mc_c4.h"

namespace {

template <bool NT>
MC_DEV void mall_load_deltas(const uint8_t *src, size_t n, size_t e0, uint32_t (&v)[C4_PER]) {
  mc_u32x4 pl[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) pl[b] = mc_ld16<NT>(src + (size_t)b * n + e0);
  c4_planes_to_deltas<MC_I2, 2>(pl, v);
}

template <bool REV, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_mall_reduce2(const uint8_t *__restrict__ src,
                                                          uint64_t *__restrict__ pair_sums,
                                                          uint64_t *__restrict__ first, C4Params p) {
  __shared__ uint64_t lds[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t pair = REV ? gridDim.x - 1 - blockIdx.x : blockIdx.x;
  const size_t e0 = pair * 2 * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  uint32_t acc[2] = {0, 0};
  uint32_t v[2][C4_PER];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (e0 + h * MC_SCAN_TILE < p.n) mall_load_deltas<NT>(src, p.n, e0 + h * MC_SCAN_TILE, v[h]);
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
    first[pair] = a;
    pair_sums[pair] = (uint32_t)(a + b);
  }
}

template <bool REV, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_mall_apply(const uint8_t *__restrict__ src,
                                                        uint8_t *__restrict__ dst,
                                                        const uint64_t *__restrict__ pair_pre,
                                                        const uint64_t *__restrict__ first, C4Params p) {
  __shared__ uint32_t red[MC_BLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * 4];
  const size_t tile = REV ? gridDim.x - 1 - blockIdx.x : blockIdx.x;
  uint32_t v[C4_PER];
  const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  if (e0 < p.n) {
    mall_load_deltas<NT>(src, p.n, e0, v);
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
  uint32_t agg;
  const uint32_t excl = mc_block_excl_scan32(run, red, &agg);
  const uint32_t tile_pre = (uint32_t)pair_pre[tile >> 1] + ((tile & 1) ? (uint32_t)first[tile >> 1] : 0u);
  c4_finish<MC_F4, MC_I2>(dst, tile, v, tile_pre + excl, outb, p);
}

template <bool R_REV, bool R_NT>
void launch_reduce(unsigned g, const uint8_t *s, uint64_t *pair, uint64_t *first, const C4Params &p,
                   hipStream_t st) {
  k_mall_reduce2<R_REV, R_NT><<<g, MC_BLOCK, 0, st>>>(s, pair, first, p);
}
template <bool A_REV, bool A_NT>
void launch_apply(unsigned g, const uint8_t *s, uint8_t *d, const uint64_t *pre, const uint64_t *first,
                  const C4Params &p, hipStream_t st) {
  k_mall_apply<A_REV, A_NT><<<g, MC_BLOCK, 0, st>>>(s, d, pre, first, p);
}


// ---------------------------------------------------------------------------
// Two-launch decode: the scan of the tile totals is folded into the passes.
// A reduce workgroup covers R consecutive tiles (2*R 16-B loads per thread in
// flight), stores the R tile totals and adds its total into its GROUP's word
// (GT tiles per group, at most 64 groups) with ONE returning 64-bit atomic:
// word = (sum << 16) + count, on its own `tstride`-word slot of `ticket`
// (the count never carries into the sum; the sum is needed mod 2^32).  The
// group's last arriver writes gtot[g] and zeroes the word (left zero).  An
// apply workgroup takes its prefix as sum(gtot[0..g)) + sum(tile totals of
// group g before its tile) -- both loaded before its data, folded into the
// block scan's one LDS round.
// ---------------------------------------------------------------------------
template <int R, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_c4r_reduce(const uint8_t *__restrict__ src, uint32_t *ws,
                                                        uint32_t *ticket, C4Params p, size_t wg0, size_t ntiles,
                                                        unsigned GT, unsigned tstride,
                                                        size_t nt_from = ~(size_t)0) {
  __shared__ uint32_t lds[R][MC_BLOCK / 64];
  uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t t0 = (wg0 + blockIdx.x) * R;
  const size_t e0 = t0 * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  uint32_t acc[R];
  uint32_t v[R][C4_PER];
#pragma unroll
  for (int h = 0; h < R; ++h)
    if (e0 + h * MC_SCAN_TILE < p.n) {
      if (NT || t0 >= nt_from) mall_load_deltas<true>(src, p.n, e0 + h * MC_SCAN_TILE, v[h]);
      else mall_load_deltas<false>(src, p.n, e0 + h * MC_SCAN_TILE, v[h]);
    }
#pragma unroll
  for (int h = 0; h < R; ++h) {
    acc[h] = 0;
    if (e0 + h * MC_SCAN_TILE < p.n) {
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) acc[h] += v[h][k];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int h = 0; h < R; ++h) acc[h] += __shfl_xor(acc[h], off, 64);
  if (lane == 0)
#pragma unroll
    for (int h = 0; h < R; ++h) lds[h][wave] = acc[h];
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t tot = 0;
#pragma unroll
  for (int h = 0; h < R; ++h) {
    uint32_t a = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) a += lds[h][w];
    if (t0 + h < ntiles) tile_tot[t0 + h] = a;
    tot += a;
  }
  const size_t g = t0 / GT;
  const size_t wgs_in_group = ((ntiles - g * GT < GT ? ntiles - g * GT : GT) + R - 1) / R;
  unsigned long long *word = reinterpret_cast<unsigned long long *>(ticket + (size_t)tstride * g);
  const unsigned long long old = atomicAdd(word, ((unsigned long long)tot << 16) | 1ull);
  if ((old & 0xffffu) + 1u == wgs_in_group) {
    gtot[g] = (uint32_t)(old >> 16) + tot;
    *word = 0;
  }
}

template <bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_c4r_apply(const uint8_t *__restrict__ src,
                                                       uint8_t *__restrict__ dst, const uint32_t *ws,
                                                       C4Params p, size_t tile0, size_t ntiles, unsigned GT,
                                                       size_t nt_from = ~(size_t)0) {
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * 4];
  const uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const size_t tile = tile0 + blockIdx.x;
  const size_t g = tile / GT, gt0 = g * GT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // prefix pieces first (their loads overlap the data loads below)
  uint32_t x = (wave == 0 && (size_t)lane < g) ? gtot[lane] : 0u;
  for (unsigned j = threadIdx.x; j < GT; j += MC_BLOCK)
    if (gt0 + j < tile) x += tile_tot[gt0 + j];
  uint32_t v[C4_PER];
  const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  if (e0 < p.n) {
    if (NT || tile >= nt_from) mall_load_deltas<true>(src, p.n, e0, v);
    else mall_load_deltas<false>(src, p.n, e0, v);
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
  c4_finish<MC_F4, MC_I2>(dst, tile, v, pre + (incl - run), outb, p);
}

template <bool NT>
void launch_c4r_reduce(int R, unsigned grid, const uint8_t *s, uint32_t *ws, uint32_t *ticket, const C4Params &p,
                       size_t wg0, size_t ntiles, unsigned GT, unsigned ts, hipStream_t st) {
  if (R == 2) k_c4r_reduce<2, NT><<<grid, MC_BLOCK, 0, st>>>(s, ws, ticket, p, wg0, ntiles, GT, ts);
  else if (R == 4) k_c4r_reduce<4, NT><<<grid, MC_BLOCK, 0, st>>>(s, ws, ticket, p, wg0, ntiles, GT, ts);
  else k_c4r_reduce<8, NT><<<grid, MC_BLOCK, 0, st>>>(s, ws, ticket, p, wg0, ntiles, GT, ts);
}

// ---------------------------------------------------------------------------
// ONE-launch decode with a lag: workgroup w reduces tile pair w and then
// applies tile pair w - LAG.  The pair it applies was reduced LAG workgroups
// earlier (in dispatch order), so its encoded planes were read ~LAG * 16 KiB
// ago: an Infinity-Cache hit while LAG * 48 KiB of traffic stays well under
// 256 MiB; and every total the apply needs (the groups before its own, the
// earlier tiles of its group) was published by workgroups dispatched before
// it.  Totals are published as 64-bit words (epoch << 32) | total in a
// persistent per-stream state buffer (zeroed once; `epoch` differs per
// call), so nothing needs resetting and stale words never match.  A wait
// past the spin bound (a predecessor not yet dispatched: never with in-order
// dispatch) falls back to computing the missing tile totals from the data.
// ---------------------------------------------------------------------------
MC_DEV uint32_t c41_tile_total_from_data(const uint8_t *src, const C4Params &p, size_t tile, uint32_t *red) {
  // block-wide sum of one tile's deltas (fallback only)
  uint32_t v[C4_PER];
  const size_t e0 = tile * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  uint32_t a = 0;
  if (e0 < p.n) {
    mall_load_deltas<false>(src, p.n, e0, v);
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) a += v[k];
  }
  uint32_t tot;
  (void)mc_block_excl_scan32(a, red, &tot);
  return tot;
}

template <int SPINS>
MC_DEV bool c41_wait(const unsigned long long *w, uint32_t epoch, uint32_t &val) {
  for (int i = 0; i < SPINS; ++i) {
    const unsigned long long x = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(x >> 32) == epoch) {
      val = (uint32_t)x;
      return true;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

__global__ __launch_bounds__(MC_BLOCK) void k_c41_decode(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                        unsigned long long *state, uint32_t *ticket, C4Params p,
                                                        size_t ntiles, size_t npairs, unsigned GT, unsigned lag,
                                                        uint32_t epoch) {
  __shared__ uint32_t lds[2][MC_BLOCK / 64];
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  __shared__ uint32_t fb[1];
  __shared__ __attribute__((aligned(16))) uint8_t outb[MC_SCAN_TILE * 4];
  unsigned long long *tile_st = state, *grp_st = state + ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t w = blockIdx.x;
  const bool do_reduce = w < npairs, do_apply = w >= lag;
  const size_t q = do_apply ? w - lag : 0;
  // every load of both halves issued up front: the reduce pair's planes and
  // the apply pair's (8 x 16 B per thread in flight)
  uint32_t rv[2][C4_PER], av[2][C4_PER];
  const size_t re0 = 2 * w * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
  const size_t ae0 = 2 * q * MC_SCAN_TILE + (size_t)threadIdx.x * C4_PER;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (do_reduce && re0 + h * MC_SCAN_TILE < p.n) mall_load_deltas<false>(src, p.n, re0 + h * MC_SCAN_TILE, rv[h]);
    if (do_apply && ae0 + h * MC_SCAN_TILE < p.n) {
      mall_load_deltas<false>(src, p.n, ae0 + h * MC_SCAN_TILE, av[h]);
    } else {
#pragma unroll
      for (int k = 0; k < C4_PER; ++k) av[h][k] = 0;
    }
  }
  // ---- reduce pair w
  if (do_reduce) {
    const size_t t0 = 2 * w;
    uint32_t acc[2] = {0, 0};
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (re0 + h * MC_SCAN_TILE < p.n) {
#pragma unroll
        for (int k = 0; k < C4_PER; ++k) acc[h] += rv[h][k];
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
      uint32_t tot = 0;
      for (int h = 0; h < 2; ++h) {
        uint32_t a = 0;
        for (int qq = 0; qq < MC_BLOCK / 64; ++qq) a += lds[h][qq];
        if (t0 + h < ntiles)
          __hip_atomic_store(tile_st + t0 + h, ((unsigned long long)epoch << 32) | a, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        tot += a;
      }
      const size_t g = t0 / GT;
      const size_t in_group = ntiles - g * GT < GT ? ntiles - g * GT : GT;
      const unsigned long long arrivals = (in_group + 1) / 2;
      unsigned long long *word = reinterpret_cast<unsigned long long *>(ticket + (size_t)MC_ARRIVAL_LINE * g);
      const unsigned long long old = atomicAdd(word, ((unsigned long long)tot << 16) | 1ull);
      if ((old & 0xffffu) + 1u == arrivals) {
        __hip_atomic_store(grp_st + g, ((unsigned long long)epoch << 32) | (uint32_t)((uint32_t)(old >> 16) + tot),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *word = 0;
      }
    }
  }
  if (!do_apply) return;
  // ---- apply pair q = w - lag (both tiles)
  const size_t g = (2 * q) / GT, gt0 = g * GT;
  for (int h = 0; h < 2; ++h) {
    const size_t tile = 2 * q + h;
    if (tile >= ntiles) break;
    uint32_t x = 0;
    bool ok = true;
    if (wave == 0 && (size_t)lane < g) ok = c41_wait<4096>(grp_st + lane, epoch, x);
    for (unsigned j = threadIdx.x; j < GT && gt0 + j < tile; j += MC_BLOCK) {
      uint32_t y = 0;
      ok = c41_wait<4096>(tile_st + gt0 + j, epoch, y) && ok;
      x += y;
    }
    if (threadIdx.x == 0) fb[0] = 0;
    __syncthreads();
    if (!ok) atomicOr(&fb[0], 1u);
    __syncthreads();
    if (fb[0]) {  // fallback: the whole prefix from the data (never expected)
      x = 0;
      uint32_t tot = 0;
      for (size_t t = 0; t < tile; ++t) tot += c41_tile_total_from_data(src, p, t, red[0]);
      if (threadIdx.x == 0) x = tot;
    }
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < C4_PER; ++k) {
      run += av[h][k];
      av[h][k] = run;
    }
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
    for (int ww = 0; ww < MC_BLOCK / 64; ++ww) {
      if (ww < wave) pre += red[0][ww];
      pre += red[1][ww];
    }
    c4_finish<MC_F4, MC_I2>(dst, tile, av[h], pre + (incl - run), outb, p);
    __syncthreads();  // outb and red are reused by the second tile
  }
}

}  // namespace

extern "C" {

// FSO(f4 <- i2) <- Delta(i2) <- Shuffle(2) decode of n elements with the
// pass orders / load policies of `flags` (above); workspace as for
// mc_fso_delta_shuffle_decode.
int mc_lab_c4_decode_mall(const void *src, void *dst, size_t n, double scale, double offset, void *workspace,
                          size_t workspace_bytes, int flags, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, MC_F4, MC_I2)) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_fso_delta_shuffle_decode_workspace(n)) return MC_ENOSPC;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t npairs = (ntiles + 1) / 2;
  uint64_t *sums = static_cast<uint64_t *>(workspace);
  uint64_t *pair = sums, *first = sums + npairs, *pre = sums + 2 * npairs;
  const unsigned gp = (unsigned)npairs, gt = (unsigned)ntiles;
  switch (flags & 3) {  // bit 1 set = temporal = NT false
    case 0: launch_reduce<false, true>(gp, s, pair, first, p, st); break;
    case 1: launch_reduce<true, true>(gp, s, pair, first, p, st); break;
    case 2: launch_reduce<false, false>(gp, s, pair, first, p, st); break;
    default: launch_reduce<true, false>(gp, s, pair, first, p, st); break;
  }
  mc_launch_scan_sums_mw<false>(pair, pre, npairs, st);
  switch ((flags >> 2) & 3) {  // bit 2 = temporal, bit 3 = reverse
    case 0: launch_apply<false, true>(gt, s, d, pre, first, p, st); break;
    case 1: launch_apply<false, false>(gt, s, d, pre, first, p, st); break;
    case 2: launch_apply<true, true>(gt, s, d, pre, first, p, st); break;
    default: launch_apply<true, false>(gt, s, d, pre, first, p, st); break;
  }
  return mc_last_launch();
}

// Two-launch decode (above) in `nslabs` slabs; flags: bit 1 reduce with
// default-policy loads, bit 2 apply with default-policy loads, bits 4-5
// log2(R) (0 -> R = 4), bits 8-: the group words' stride in uint32 words
// (0 -> one 128-B line).  `ticket`: 64 strides of zeroed words, left zero.
size_t mc_lab_c4_2l_workspace(size_t n) {  // tile totals + 64 group totals
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  return (ntiles + 64) * sizeof(uint32_t);
}

int mc_lab_c4_decode_2l(const void *src, void *dst, size_t n, double scale, double offset, void *workspace,
                        size_t workspace_bytes, uint32_t *ticket, int flags, int nslabs, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, MC_F4, MC_I2) || !ticket || nslabs < 1) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_lab_c4_2l_workspace(n)) return MC_ENOSPC;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const int lr = (flags >> 4) & 3;
  const int R = lr ? 1 << lr : 4;
  unsigned GT = 256;  // tiles per group: at most 64 groups, at most 1024 tiles per group
  while ((ntiles + GT - 1) / GT > 64) GT *= 2;
  if (GT > 1024) return MC_EINVAL;
  const size_t ngroups = (ntiles + GT - 1) / GT;
  const unsigned ts = (flags >> 8) ? (unsigned)(flags >> 8) : MC_ARRIVAL_LINE;
  uint32_t *ws = static_cast<uint32_t *>(workspace);
  for (int sl = 0; sl < nslabs; ++sl) {
    const size_t g0 = ngroups * sl / nslabs, g1 = ngroups * (sl + 1) / nslabs;
    if (g1 == g0) continue;
    const size_t t0 = g0 * GT, t1 = g1 * GT < ntiles ? g1 * GT : ntiles;
    const unsigned grid = (unsigned)((t1 - t0 + R - 1) / R);
    if (flags & 2) launch_c4r_reduce<false>(R, grid, s, ws, ticket, p, t0 / R, ntiles, GT, ts, st);
    else launch_c4r_reduce<true>(R, grid, s, ws, ticket, p, t0 / R, ntiles, GT, ts, st);
    if (flags & 4) k_c4r_apply<false><<<(unsigned)(t1 - t0), MC_BLOCK, 0, st>>>(s, d, ws, p, t0, ntiles, GT);
    else k_c4r_apply<true><<<(unsigned)(t1 - t0), MC_BLOCK, 0, st>>>(s, d, ws, p, t0, ntiles, GT);
  }
  return mc_last_launch();
}

// Two-stream slab pipeline: the reduce pass of slab k runs on `stream`, the
// apply pass of slab k on `side` once reduce k is done, so reduce k+1 overlaps
// apply k (no drained chip between slabs) and apply k re-reads planes read one
// slab earlier (an Infinity-Cache hit while ~2 slabs of traffic fit in it).
// window > 0: reduce k waits for apply k - window (bounds the reuse distance).
// Slabs are whole groups, as in mc_lab_c4_decode_2l.  flags as there.
int mc_lab_c4_decode_2s(const void *src, void *dst, size_t n, double scale, double offset, void *workspace,
                        size_t workspace_bytes, uint32_t *ticket, int flags, int nslabs, int window,
                        mc_stream_t stream, mc_stream_t side) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, MC_F4, MC_I2) || !ticket || nslabs < 1 || nslabs > 64) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_lab_c4_2l_workspace(n)) return MC_ENOSPC;
  static hipEvent_t ev[2 * 64 + 1];
  static bool init = false;
  if (!init) {
    for (auto &e : ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return MC_EHIP_BASE - 1;
    init = true;
  }
  hipEvent_t *ev_r = ev, *ev_a = ev + 64, ev0 = ev[128];
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream, sd = (hipStream_t)side;
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const int lr = (flags >> 4) & 3;
  const int R = lr ? 1 << lr : 4;
  unsigned GT = 256;
  while ((ntiles + GT - 1) / GT > 64) GT *= 2;
  if (GT > 1024) return MC_EINVAL;
  const size_t ngroups = (ntiles + GT - 1) / GT;
  uint32_t *ws = static_cast<uint32_t *>(workspace);
  (void)hipEventRecord(ev0, st);
  (void)hipStreamWaitEvent(sd, ev0, 0);
  int last = -1;
  for (int sl = 0; sl < nslabs; ++sl) {
    const size_t g0 = ngroups * sl / nslabs, g1 = ngroups * (sl + 1) / nslabs;
    if (g1 == g0) continue;
    const size_t t0 = g0 * GT, t1 = g1 * GT < ntiles ? g1 * GT : ntiles;
    if (window > 0 && sl >= window) (void)hipStreamWaitEvent(st, ev_a[sl - window], 0);
    const unsigned grid = (unsigned)((t1 - t0 + R - 1) / R);
    if (flags & 2) launch_c4r_reduce<false>(R, grid, s, ws, ticket, p, t0 / R, ntiles, GT, MC_ARRIVAL_LINE, st);
    else launch_c4r_reduce<true>(R, grid, s, ws, ticket, p, t0 / R, ntiles, GT, MC_ARRIVAL_LINE, st);
    (void)hipEventRecord(ev_r[sl], st);
    (void)hipStreamWaitEvent(sd, ev_r[sl], 0);
    if (flags & 4) k_c4r_apply<false><<<(unsigned)(t1 - t0), MC_BLOCK, 0, sd>>>(s, d, ws, p, t0, ntiles, GT);
    else k_c4r_apply<true><<<(unsigned)(t1 - t0), MC_BLOCK, 0, sd>>>(s, d, ws, p, t0, ntiles, GT);
    (void)hipEventRecord(ev_a[sl], sd);
    last = sl;
  }
  if (last >= 0) (void)hipStreamWaitEvent(st, ev_a[last], 0);
  return mc_last_launch();
}

// Two-launch decode (R = 2, one slab) with a per-tile load policy: the
// reduce pass loads tiles >= r_nt_from nontemporally (default policy before),
// the apply pass tiles >= a_nt_from.  The apply pass re-reads from the
// Infinity Cache only what stayed there; tiles that would be evicted anyway
// are read nt so they neither slow the reduce pass nor displace the others.
int mc_lab_c4_decode_split(const void *src, void *dst, size_t n, double scale, double offset, void *workspace,
                           size_t workspace_bytes, uint32_t *ticket, size_t r_nt_from, size_t a_nt_from,
                           mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, MC_F4, MC_I2) || !ticket) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_lab_c4_2l_workspace(n)) return MC_ENOSPC;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  unsigned GT = 256;
  while ((ntiles + GT - 1) / GT > 64) GT *= 2;
  if (GT > 1024) return MC_EINVAL;
  uint32_t *ws = static_cast<uint32_t *>(workspace);
  k_c4r_reduce<2, false><<<(unsigned)((ntiles + 1) / 2), MC_BLOCK, 0, st>>>(s, ws, ticket, p, 0, ntiles, GT,
                                                                           MC_ARRIVAL_LINE, r_nt_from);
  k_c4r_apply<false><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, ws, p, 0, ntiles, GT, a_nt_from);
  return mc_last_launch();
}

// One-launch lag decode (above).  state: (ntiles + 64) 64-bit words, zeroed
// once and kept per stream; epoch: a different nonzero value per call;
// ticket: MC_ARRIVAL_WORDS zeroed words, left zero; lag in tile pairs.
size_t mc_lab_c41_state_bytes(size_t n) {
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  return (ntiles + 64) * 8;
}

int mc_lab_c4_decode_1l(const void *src, void *dst, size_t n, double scale, double offset, void *state,
                        size_t state_bytes, uint32_t *ticket, unsigned lag, uint32_t epoch, mc_stream_t stream) {
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, MC_F4, MC_I2) || !ticket || !epoch || lag == 0) return MC_EINVAL;
  if (!state || state_bytes < mc_lab_c41_state_bytes(n)) return MC_ENOSPC;
  const C4Params p = c4_decode_params(n, scale, offset);
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t npairs = (ntiles + 1) / 2;
  unsigned GT = 256;
  while ((ntiles + GT - 1) / GT > 64) GT *= 2;
  if (GT > 1024) return MC_EINVAL;
  k_c41_decode<<<(unsigned)(npairs + lag), MC_BLOCK, 0, (hipStream_t)stream>>>(
      static_cast<const uint8_t *>(src), static_cast<uint8_t *>(dst), static_cast<unsigned long long *>(state),
      ticket, p, ntiles, npairs, GT, lag, epoch);
  return mc_last_launch();
}

}  // extern "C"
