// mc_scan.hip -- Delta decode = np.cumsum(enc, out=dec) (delta.py:69-83).
//
// numpy accumulates in the output dtype (add.accumulate with otype = dtype):
//   * integer dtypes: wrap-around addition, associative, so a parallel scan is
//     bit-exact.  Three passes over 4096-element tiles: per-tile totals
//     (k_scan_reduce), an exclusive scan of the totals staged through LDS by
//     one workgroup (k_scan_sums), then every tile rescanned with its prefix
//     (k_scan_apply: lane-serial over 4 elements, wave __shfl_up scan, LDS
//     across the 4 waves).  Lanes read 4 consecutive elements with one vector
//     access; the tile loop is 4 steps of 4x256 elements.
//   * bool: numpy's bool add loop is logical or -- also associative.
//   * float dtypes: numpy adds left to right with a rounding after every add;
//     no reassociation reproduces that, so the float path keeps the serial
//     order exactly (k_scan_serial: one dependent add chain per chunk fed
//     through double-buffered LDS by a second wave).  Bit-exact; a single
//     chunk runs at the latency of one add per element, batches
//     run one chain per workgroup.
//   * batches of chunks (mc_delta_decode_batch): one workgroup per chunk with
//     a running carry (k_scan_rows), single pass.
#include "mc_scan.h"

#include <stdlib.h>

#include <type_traits>

namespace {

// 4 consecutive elements i0..i0+3 of dtype a (as accumulation values in d)
template <int A_, int D_, bool VEC>
MC_DEV void load4_acc(const uint8_t *src, size_t i0, size_t n, int a, int d, uint64_t (&v)[4],
                      int &cnt) {
  const int as = mc_itemsize(a);
  if (VEC && i0 + 4 <= n) {
    uint64_t e[4];
    mc_load4(src + i0 * as, as, e);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (uint64_t)mc_num_cast(mc_num_from_bits(e[k], a), a, d).i;
    cnt = 4;
  } else {
    cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = 0;
      if (i0 + k < n) {
        v[k] = (uint64_t)mc_num_cast(mc_num_from_bits(mc_load_elem_u(src, i0 + k, as), a), a, d).i;
        cnt = k + 1;
      }
    }
  }
}

template <bool OR_OP, int A_, int D_, bool VEC>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_reduce(const uint8_t *__restrict__ src,
                                                          size_t n, int a_rt, int d_rt,
                                                          uint64_t *__restrict__ sums) {
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const int a = A_ >= 0 ? A_ : a_rt, d = D_ >= 0 ? D_ : d_rt;
  const size_t base = (size_t)blockIdx.x * MC_SCAN_TILE;
  uint64_t acc = 0;
#pragma unroll
  for (int s = 0; s < MC_SCAN_STEPS; ++s) {
    const size_t i0 = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    uint64_t v[4];
    int cnt;
    load4_acc<A_, D_, VEC>(src, i0, n, a, d, v, cnt);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = mc_scan_combine<OR_OP>(acc, v[k]);
  }
  uint64_t tot;
  mc_block_excl_scan<OR_OP>(acc, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <bool OR_OP, int A_, int D_, bool VEC>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_apply(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t n,
                                                         int a_rt, int d_rt,
                                                         const uint64_t *__restrict__ sums) {
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const int a = A_ >= 0 ? A_ : a_rt, d = D_ >= 0 ? D_ : d_rt;
  const int ds = mc_itemsize(d);
  const size_t base = (size_t)blockIdx.x * MC_SCAN_TILE;
  uint64_t carry = sums[blockIdx.x];
#pragma unroll
  for (int s = 0; s < MC_SCAN_STEPS; ++s) {
    const size_t i0 = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    uint64_t v[4];
    int cnt;
    load4_acc<A_, D_, VEC>(src, i0, n, a, d, v, cnt);
    uint64_t p[4];
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      run = mc_scan_combine<OR_OP>(run, v[k]);
      p[k] = run;
    }
    uint64_t tot;
    const uint64_t excl = mc_block_excl_scan<OR_OP>(run, lds, &tot);
    const uint64_t pre = mc_scan_combine<OR_OP>(carry, excl);
    uint64_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = mc_to_storage((uint64_t)mc_wrap((int64_t)mc_scan_combine<OR_OP>(pre, p[k]), d), d);
    if (VEC && cnt == 4) {
      mc_store4(dst + i0 * ds, ds, o);
    } else {
      for (int k = 0; k < cnt; ++k) mc_store_elem_u(dst, i0 + k, ds, o[k]);
    }
    carry = mc_scan_combine<OR_OP>(carry, tot);
  }
}

// ---------------------------------------------------------------------------
// integer / bool Delta decode of a batch of chunks: one workgroup per chunk
// walks its chunk in 4096-element tiles with a running carry (single pass,
// no workspace).  The next tile's loads are issued before the current tile's
// block scans, so each workgroup keeps 2 tiles of reads in flight; thousands
// of chunks fill the chip.  (A single large chunk uses the 3-pass scan.)
// ---------------------------------------------------------------------------
template <bool OR_OP, int A_, int D_, bool VEC>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_rows(const uint8_t *__restrict__ src,
                                                        size_t src_stride,
                                                        uint8_t *__restrict__ dst,
                                                        size_t dst_stride, size_t n, int a_rt,
                                                        int d_rt) {
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const int a = A_ >= 0 ? A_ : a_rt, d = D_ >= 0 ? D_ : d_rt;
  const int ds = mc_itemsize(d);
  src += (size_t)blockIdx.x * src_stride;
  dst += (size_t)blockIdx.x * dst_stride;
  uint64_t carry = 0;
  uint64_t v[MC_SCAN_STEPS][4];
  int cnt[MC_SCAN_STEPS];
  auto load_tile = [&](size_t base) {
#pragma unroll
    for (int s = 0; s < MC_SCAN_STEPS; ++s)
      load4_acc<A_, D_, VEC>(src, base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x, n, a,
                             d, v[s], cnt[s]);
  };
  if (n) load_tile(0);
  for (size_t base = 0; base < n; base += MC_SCAN_TILE) {
    uint64_t cur[MC_SCAN_STEPS][4];
    int ccnt[MC_SCAN_STEPS];
#pragma unroll
    for (int s = 0; s < MC_SCAN_STEPS; ++s) {
      ccnt[s] = cnt[s];
#pragma unroll
      for (int k = 0; k < 4; ++k) cur[s][k] = v[s][k];
    }
    if (base + MC_SCAN_TILE < n) load_tile(base + MC_SCAN_TILE);
#pragma unroll
    for (int s = 0; s < MC_SCAN_STEPS; ++s) {
      const size_t i0 = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
      uint64_t p[4];
      uint64_t run = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        run = mc_scan_combine<OR_OP>(run, cur[s][k]);
        p[k] = run;
      }
      uint64_t tot;
      const uint64_t excl = mc_block_excl_scan<OR_OP>(run, lds, &tot);
      const uint64_t pre = mc_scan_combine<OR_OP>(carry, excl);
      uint64_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = mc_to_storage((uint64_t)mc_wrap((int64_t)mc_scan_combine<OR_OP>(pre, p[k]), d), d);
      if (VEC && ccnt[s] == 4) {
        mc_store4(dst + i0 * ds, ds, o);
      } else {
        for (int k = 0; k < ccnt[s]; ++k) mc_store_elem_u(dst, i0 + k, ds, o[k]);
      }
      carry = mc_scan_combine<OR_OP>(carry, tot);
    }
  }
}

template <bool OR_OP, int A_, int D_, bool VEC>
static void launch_rows(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n, size_t rows,
                        int a, int dt, hipStream_t st) {
  k_scan_rows<OR_OP, A_, D_, VEC><<<(unsigned)rows, MC_BLOCK, 0, st>>>(s, ss, d, dss, n, a, dt);
}

template <bool OR_OP, int A_, int D_, bool VEC>
static void launch_int_scan(const uint8_t *s, uint8_t *d, size_t n, int a, int dt, uint64_t *sums,
                            size_t ntiles, hipStream_t st) {
  k_scan_reduce<OR_OP, A_, D_, VEC><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, n, a, dt, sums);
  mc_launch_scan_sums<OR_OP>(sums, ntiles, st);
  k_scan_apply<OR_OP, A_, D_, VEC><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, a, dt, sums);
}

// ---------------------------------------------------------------------------
// Fast path for same-width integer Delta decode (astype == dtype, 16-B
// aligned): a thread owns 32 consecutive bytes (DS_PER = 32/ES elements: two
// 16-B vectors), so a tile of DS_PER * 256 elements (8 KiB) needs one block
// scan, and the reduce pass covers groups of DS_GROUP tiles (32 KiB per
// workgroup, all loads in flight at once) so that the tile-total scan runs
// over groups only: tile t's prefix = group_pre[t / DS_GROUP] + part[t], with
// part[t] the sum of the tiles before t in its group.  Arithmetic is modular
// on the raw bits (mod 2^32 for ES <= 4, wrapped to the dtype width by the
// store) -- exactly numpy's wrapping add.
// ---------------------------------------------------------------------------
constexpr int DS_GROUP = 4;

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

template <int ES>
using dacc_t = typename std::conditional<ES == 8, uint64_t, uint32_t>::type;

template <int ES>
constexpr int ds_per() { return 32 / ES; }
template <int ES>
constexpr size_t ds_tile() { return (size_t)ds_per<ES>() * MC_BLOCK; }

// the values of elements [e0, e0 + PER/2) (one 16-B vector; zeros past n)
// into v[at .. at + PER/2)
// BE: big-endian elements (bytes reversed after the load, v_perm_b32)
template <int ES, bool NT = true, bool BE = false>
MC_DEV void ds_load_half(const uint8_t *src, size_t n, size_t e0, dacc_t<ES> (&v)[ds_per<ES>()], int at) {
  constexpr int H = ds_per<ES>() / 2;
  if (e0 + H <= n) {
    mc_u32x4 w = mc_ld16<NT>(src + e0 * ES);
    if constexpr (BE) w = mc_bswap_vec<ES>(w);
    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < H; ++i) {
      if constexpr (ES == 1) v[at + i] = (d[i >> 2] >> (8 * (i & 3))) & 0xffu;
      else if constexpr (ES == 2) v[at + i] = (d[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      else if constexpr (ES == 4) v[at + i] = d[i];
      else v[at + i] = ((uint64_t)d[2 * i + 1] << 32) | d[2 * i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < H; ++i)
      v[at + i] = e0 + i < n ? (dacc_t<ES>)(BE ? mc_bswap_n(mc_load_elem(src, e0 + i, ES), ES) : mc_load_elem(src, e0 + i, ES))
                             : 0;
  }
}


template <int ES, bool BE = false>
__global__ __launch_bounds__(MC_BLOCK) void k_dscan_reduce(const uint8_t *__restrict__ src, size_t n,
                                                          uint64_t *__restrict__ group_sums,
                                                          uint64_t *__restrict__ part) {
  constexpr int PER = ds_per<ES>();
  constexpr size_t TE = ds_tile<ES>();
  __shared__ uint64_t lds[DS_GROUP][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t t0 = (size_t)blockIdx.x * DS_GROUP;  // first tile of the group
  // a tile total does not depend on which thread adds which element, so the
  // loads are lane-contiguous 16-B vectors (each wave instruction covers 1 KiB
  // contiguously) instead of the apply pass's 32 B per thread: half of tile h
  // at 16*tid and the other half 16*MC_BLOCK bytes later.  Totals are only
  // needed mod 2^(8*ES), so bytes and halfwords are summed per dword with
  // v_dot4_u32_u8 / v_dot2_u32_u16 instead of one extract + add per element.
  uint64_t acc[DS_GROUP];
  if ((t0 + DS_GROUP) * TE <= n) {
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) {
      const uint8_t *tb = src + (t0 + h) * TE * ES;
      mc_u32x4 w0 = mc_ld16<true>(tb + 16 * (size_t)threadIdx.x);
      mc_u32x4 w1 = mc_ld16<true>(tb + 16 * (size_t)(MC_BLOCK + threadIdx.x));
      if constexpr (BE) {
        w0 = mc_bswap_vec<ES>(w0);
        w1 = mc_bswap_vec<ES>(w1);
      }
      const uint32_t d[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      if constexpr (ES == 8) {
        uint64_t a = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) a += ((uint64_t)d[2 * i + 1] << 32) | d[2 * i];
        acc[h] = a;
      } else {
        uint32_t a = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if constexpr (ES == 1) a = __builtin_amdgcn_udot4(d[i], 0x01010101u, a, false);
          else if constexpr (ES == 2) a = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, d[i]), ushort2_t{1, 1}, a, false);
          else a += d[i];
        }
        acc[h] = a;
      }
    }
  } else {
    constexpr int HALF = PER / 2;
    dacc_t<ES> v[DS_GROUP][PER];
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) {
      const size_t tb = (t0 + h) * TE;
      ds_load_half<ES, true, BE>(src, n, tb + (size_t)threadIdx.x * HALF, v[h], 0);
      ds_load_half<ES, true, BE>(src, n, tb + (size_t)(MC_BLOCK + threadIdx.x) * HALF, v[h], HALF);
    }
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) {
      acc[h] = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i) acc[h] += v[h][i];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) acc[h] += __shfl_xor(acc[h], off, 64);
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) lds[h][wave] = acc[h];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (int h = 0; h < DS_GROUP; ++h) {
      uint64_t tot = 0;
      for (int w = 0; w < MC_BLOCK / 64; ++w) tot += lds[h][w];
      part[t0 + h] = run;  // part[] has DS_GROUP * ngroups entries
      run += tot;
    }
    group_sums[blockIdx.x] = run;
  }
}

// elements [e0, e0 + PER/2) from v[at ..] (one 16-B vector; nothing past n)
template <int ES, bool BE = false>
MC_DEV void ds_store_half(uint8_t *dst, size_t n, size_t e0, const dacc_t<ES> (&v)[ds_per<ES>()], int at) {
  constexpr int H = ds_per<ES>() / 2;
  if (e0 + H <= n) {
    uint32_t d[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < H; ++i) {
      if constexpr (ES == 1) d[i >> 2] |= ((uint32_t)v[at + i] & 0xffu) << (8 * (i & 3));
      else if constexpr (ES == 2) d[i >> 1] |= ((uint32_t)v[at + i] & 0xffffu) << (16 * (i & 1));
      else if constexpr (ES == 4) d[i] = (uint32_t)v[at + i];
      else { d[2 * i] = (uint32_t)v[at + i]; d[2 * i + 1] = (uint32_t)((uint64_t)v[at + i] >> 32); }
    }
    mc_u32x4 w = mc_u32x4{d[0], d[1], d[2], d[3]};
    if constexpr (BE) w = mc_bswap_vec<ES>(w);
    mc_st16<true>(dst + e0 * ES, w);
  } else {
    for (int i = 0; i < H && e0 + i < n; ++i)
      mc_store_elem(dst, e0 + i, ES, BE ? mc_bswap_n((uint64_t)v[at + i], ES) : (uint64_t)v[at + i]);
  }
}

// exclusive block scans of two per-thread values at once (the two halves of
// a tile), modulo 2^(8 * sizeof(T)), one LDS round (one __syncthreads; a
// caller that loops alternates two `lds` buffers); tot_a / tot_b = totals
template <typename T>
MC_DEV void ds_block_scan2(T a, T b, T (&lds)[2][MC_BLOCK / 64], T &ea, T &eb, T &tot_a, T &tot_b) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T ia = a, ib = b;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T oa = __shfl_up(ia, off, 64), ob = __shfl_up(ib, off, 64);
    if (lane >= off) {
      ia += oa;
      ib += ob;
    }
  }
  if (lane == 63) {
    lds[0][wave] = ia;
    lds[1][wave] = ib;
  }
  __syncthreads();
  T pa = 0, pb = 0, ta = 0, tb = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) {
    const T xa = lds[0][w], xb = lds[1][w];
    if (w < wave) {
      pa += xa;
      pb += xb;
    }
    ta += xa;
    tb += xb;
  }
  const T ua = __shfl_up(ia, 1, 64), ub = __shfl_up(ib, 1, 64);
  ea = pa + (lane ? ua : (T)0);
  eb = pb + (lane ? ub : (T)0);
  tot_a = ta;
  tot_b = tb;
}

// Scan of one tile with lane-contiguous 16-B accesses: thread t owns the
// vector at 16*t of each half of the tile (half A = the first 16*MC_BLOCK
// bytes, half B = the rest), scans both in registers, and one two-value
// block scan gives every vector its prefix (B's offset by A's total).  Each
// wave load/store instruction covers 1 KiB contiguously (the 32-B-per-thread
// layout touched 2 KiB with gaps per instruction).
template <int ES, bool BE = false>
__global__ __launch_bounds__(MC_BLOCK) void k_dscan_apply(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t n,
                                                         const uint64_t *__restrict__ group_pre,
                                                         const uint64_t *__restrict__ part) {
  constexpr int PER = ds_per<ES>();
  constexpr int H = PER / 2;
  using T = dacc_t<ES>;
  __shared__ T lds[2][MC_BLOCK / 64];
  const size_t tile = blockIdx.x;
  const size_t ea0 = tile * ds_tile<ES>() + (size_t)threadIdx.x * H;
  const size_t eb0 = tile * ds_tile<ES>() + (size_t)(MC_BLOCK + threadIdx.x) * H;
  T v[PER];
  ds_load_half<ES, true, BE>(src, n, ea0, v, 0);
  ds_load_half<ES, true, BE>(src, n, eb0, v, H);
  T ra = 0, rb = 0;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    ra += v[i];
    v[i] = ra;
    rb += v[H + i];
    v[H + i] = rb;
  }
  T xa, xb, ta, tb;
  ds_block_scan2<T>(ra, rb, lds, xa, xb, ta, tb);
  const T pre = (T)(group_pre[tile / DS_GROUP] + part[tile]);
  const T pa = pre + xa, pb = pre + ta + xb;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    v[i] += pa;
    v[H + i] += pb;
  }
  ds_store_half<ES, BE>(dst, n, ea0, v, 0);
  ds_store_half<ES, BE>(dst, n, eb0, v, H);
}

// workspace entries of the fast path: group sums, part[] (whole groups of
// tiles), group prefixes
static size_t dscan_ws_entries(size_t n, int es) {
  const size_t te = (size_t)(32 / es) * MC_BLOCK;
  const size_t ngroups = ((n + te - 1) / te + DS_GROUP - 1) / DS_GROUP;
  return ngroups * DS_GROUP + 2 * ngroups;
}

// Batched same-width integer Delta decode: one workgroup per chunk walks it in
// 8 KiB tiles with a running carry, the next tile's loads issued before the
// current tile's scan; the two-half tile layout of k_dscan_apply.
template <int ES, bool BE = false>
__global__ __launch_bounds__(MC_BLOCK) void k_dscan_rows(const uint8_t *__restrict__ src,
                                                        size_t src_stride,
                                                        uint8_t *__restrict__ dst,
                                                        size_t dst_stride, size_t n) {
  constexpr int PER = ds_per<ES>();
  constexpr int H = PER / 2;
  constexpr size_t TE = ds_tile<ES>();
  using T = dacc_t<ES>;
  __shared__ T lds[2][2][MC_BLOCK / 64];  // [iteration parity][half][wave]
  src += (size_t)blockIdx.x * src_stride;
  dst += (size_t)blockIdx.x * dst_stride;
  const size_t oa = (size_t)threadIdx.x * H, ob = (size_t)(MC_BLOCK + threadIdx.x) * H;
  T carry = 0;
  T nxt[PER];
  ds_load_half<ES, true, BE>(src, n, oa, nxt, 0);
  ds_load_half<ES, true, BE>(src, n, ob, nxt, H);
  int parity = 0;
  for (size_t base = 0; base < n; base += TE, parity ^= 1) {
    T v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = nxt[i];
    if (base + TE < n) {
      ds_load_half<ES, true, BE>(src, n, base + TE + oa, nxt, 0);
      ds_load_half<ES, true, BE>(src, n, base + TE + ob, nxt, H);
    }
    T ra = 0, rb = 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      ra += v[i];
      v[i] = ra;
      rb += v[H + i];
      v[H + i] = rb;
    }
    T xa, xb, ta, tb;
    ds_block_scan2<T>(ra, rb, lds[parity], xa, xb, ta, tb);
    const T pa = carry + xa, pb = carry + ta + xb;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      v[i] += pa;
      v[H + i] += pb;
    }
    ds_store_half<ES, BE>(dst, n, base + oa, v, 0);
    ds_store_half<ES, BE>(dst, n, base + ob, v, H);
    carry += ta + tb;
  }
}

// ---------------------------------------------------------------------------
// Two-launch same-width decode (ES <= 4, with an arrival ticket): the scan of
// the tile totals folded into the passes, as for the C4 decode (mc_c4.hip,
// k_c4_reduce_g / k_c4_apply_g).  A reduce workgroup covers DS_GROUP tiles
// (default-policy loads: the apply pass re-reads them partly from the
// Infinity Cache), stores their totals and adds its total into its group's
// word with one returning 64-bit atomic, word = (sum << 16) + count (sums
// mod 2^32 suffice for ES <= 4); the group's last arriver writes gtot[g] and
// zeroes the word.  The apply workgroup's prefix = sum(gtot[0..g)) + the
// totals of its group's earlier tiles, loaded before its data.
// ---------------------------------------------------------------------------
constexpr unsigned DS_MAX_GROUPS = 64;

static inline unsigned ds_group_tiles(size_t ntiles) {
  unsigned gt = 256;  // tiles per group (a multiple of DS_GROUP): at most 64 groups
  while ((ntiles + gt - 1) / gt > DS_MAX_GROUPS) gt *= 2;
  return gt;
}

template <int ES, bool NT = false, bool BE = false>
__global__ __launch_bounds__(MC_BLOCK) void k_dscan_reduce_g(const uint8_t *__restrict__ src, size_t n,
                                                            uint32_t *ws, uint32_t *ticket, size_t ntiles,
                                                            unsigned GT) {
  static_assert(ES <= 4, "group sums are kept mod 2^32");
  constexpr int PER = ds_per<ES>();
  constexpr size_t TE = ds_tile<ES>();
  __shared__ uint32_t lds[DS_GROUP][MC_BLOCK / 64];
  uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // (walking the tiles from the end, so that the apply pass finds its first
  // tiles among the ones read last, measured the same: 124-130 us either way
  // for 256 MiB i1/i2/i4)
  const size_t t0 = (size_t)blockIdx.x * DS_GROUP;
  uint32_t acc[DS_GROUP];
  if ((t0 + DS_GROUP) * TE <= n) {
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) {
      const uint8_t *tb = src + (t0 + h) * TE * ES;
      mc_u32x4 w0 = mc_ld16<NT>(tb + 16 * (size_t)threadIdx.x);
      mc_u32x4 w1 = mc_ld16<NT>(tb + 16 * (size_t)(MC_BLOCK + threadIdx.x));
      if constexpr (BE) {
        w0 = mc_bswap_vec<ES>(w0);
        w1 = mc_bswap_vec<ES>(w1);
      }
      const uint32_t d[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      uint32_t a = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (ES == 1) a = __builtin_amdgcn_udot4(d[i], 0x01010101u, a, false);
        else if constexpr (ES == 2) a = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, d[i]), ushort2_t{1, 1}, a, false);
        else a += d[i];
      }
      acc[h] = a;
    }
  } else {
    constexpr int HALF = PER / 2;
    dacc_t<ES> v[DS_GROUP][PER];
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) {
      const size_t tb = (t0 + h) * TE;
      ds_load_half<ES, NT, BE>(src, n, tb + (size_t)threadIdx.x * HALF, v[h], 0);
      ds_load_half<ES, NT, BE>(src, n, tb + (size_t)(MC_BLOCK + threadIdx.x) * HALF, v[h], HALF);
    }
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) {
      acc[h] = 0;
#pragma unroll
      for (int i = 0; i < PER; ++i) acc[h] += (uint32_t)v[h][i];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) acc[h] += __shfl_xor(acc[h], off, 64);
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < DS_GROUP; ++h) lds[h][wave] = acc[h];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  uint32_t tot = 0;
  for (int h = 0; h < DS_GROUP; ++h) {
    uint32_t a = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) a += lds[h][w];
    if (t0 + h < ntiles) tile_tot[t0 + h] = a;
    tot += a;
  }
  const size_t g = t0 / GT;
  const size_t in_group = ntiles - g * GT < GT ? ntiles - g * GT : GT;
  const unsigned long long arrivals = (in_group + DS_GROUP - 1) / DS_GROUP;
  unsigned long long *word = reinterpret_cast<unsigned long long *>(ticket + (size_t)MC_ARRIVAL_LINE * g);
  const unsigned long long old = atomicAdd(word, ((unsigned long long)tot << 16) | 1ull);
  if ((old & 0xffffu) + 1u == arrivals) {
    gtot[g] = (uint32_t)(old >> 16) + tot;
    *word = 0;  // every arrival of this call is in: left zero
  }
}

template <int ES, bool NT = false, bool BE = false>
__global__ __launch_bounds__(MC_BLOCK) void k_dscan_apply_g(const uint8_t *__restrict__ src,
                                                           uint8_t *__restrict__ dst, size_t n, const uint32_t *ws,
                                                           size_t ntiles, unsigned GT) {
  constexpr int PER = ds_per<ES>();
  constexpr int H = PER / 2;
  using T = dacc_t<ES>;  // uint32_t for ES <= 4
  __shared__ T lds[3][MC_BLOCK / 64];
  const uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const size_t tile = blockIdx.x;
  const size_t g = tile / GT, gt0 = g * GT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t ea0 = tile * ds_tile<ES>() + (size_t)threadIdx.x * H;
  const size_t eb0 = tile * ds_tile<ES>() + (size_t)(MC_BLOCK + threadIdx.x) * H;
  // the tile's data and its prefix words in flight together (one memory
  // round trip per workgroup): a full tile's two vectors first, with no
  // branch between them and the prefix loads, then the prefix words in
  // batches of 8 per thread.  (Loaded in the other order, each behind the
  // previous one's wait, the workgroup paid three round trips: the apply
  // pass's waves sat parked 72 % of their cycles, round 5.)
  const bool full = (tile + 1) * ds_tile<ES>() <= n;
  mc_u32x4 wa{}, wb{};
  if (full) {
    wa = mc_ld16<NT>(src + ea0 * ES);
    wb = mc_ld16<NT>(src + eb0 * ES);
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
  uint32_t x = tile_tots(0);  // GT <= 2048 (up to 128 Mi tiles): this batch only
  for (unsigned j0 = 8 * MC_BLOCK; j0 < GT; j0 += 8 * MC_BLOCK) x += tile_tots(j0);
  x += xg;
  T v[PER];
  if (full) {
    if constexpr (BE) {
      wa = mc_bswap_vec<ES>(wa);
      wb = mc_bswap_vec<ES>(wb);
    }
    const uint32_t da[4] = {wa.x, wa.y, wa.z, wa.w}, db[4] = {wb.x, wb.y, wb.z, wb.w};
#pragma unroll
    for (int i = 0; i < H; ++i) {
      if constexpr (ES == 1) {
        v[i] = (da[i >> 2] >> (8 * (i & 3))) & 0xffu;
        v[H + i] = (db[i >> 2] >> (8 * (i & 3))) & 0xffu;
      } else if constexpr (ES == 2) {
        v[i] = (da[i >> 1] >> (16 * (i & 1))) & 0xffffu;
        v[H + i] = (db[i >> 1] >> (16 * (i & 1))) & 0xffffu;
      } else {
        v[i] = da[i];
        v[H + i] = db[i];
      }
    }
  } else {
    ds_load_half<ES, NT, BE>(src, n, ea0, v, 0);
    ds_load_half<ES, NT, BE>(src, n, eb0, v, H);
  }
  T ra = 0, rb = 0;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    ra += v[i];
    v[i] = ra;
    rb += v[H + i];
    v[H + i] = rb;
  }
  // one LDS round: the two-half exclusive scan and the block sum of x
  T ia = ra, ib = rb;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T oa = __shfl_up(ia, off, 64), ob = __shfl_up(ib, off, 64);
    if (lane >= off) {
      ia += oa;
      ib += ob;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  if (lane == 63) {
    lds[0][wave] = ia;
    lds[1][wave] = ib;
  }
  if (lane == 0) lds[2][wave] = x;
  __syncthreads();
  T pa = 0, pb = 0, ta = 0, pre = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) {
    if (w < wave) {
      pa += lds[0][w];
      pb += lds[1][w];
    }
    ta += lds[0][w];
    pre += lds[2][w];
  }
  const T ua = __shfl_up(ia, 1, 64), ub = __shfl_up(ib, 1, 64);
  const T xa = pa + (lane ? ua : (T)0), xb = pb + (lane ? ub : (T)0);
  const T qa = pre + xa, qb = pre + ta + xb;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    v[i] += qa;
    v[H + i] += qb;
  }
  ds_store_half<ES, BE>(dst, n, ea0, v, 0);
  ds_store_half<ES, BE>(dst, n, eb0, v, H);
}

template <int ES, bool BE = false>
static void launch_dscan_g(const uint8_t *s, uint8_t *d, size_t n, uint32_t *ws, uint32_t *ticket, hipStream_t st) {
  const size_t ntiles = (n + ds_tile<ES>() - 1) / ds_tile<ES>();
  const unsigned gt = ds_group_tiles(ntiles);
  const unsigned rg = (unsigned)((ntiles + DS_GROUP - 1) / DS_GROUP);
  // load policy per pass, mc_sched.dscan_nt (lab A/B): bit 0 = nontemporal loads in
  // the reduce pass, bit 1 in the apply pass.  Default 2: the reduce pass
  // keeps default-policy loads (what the Infinity Cache retains serves the
  // re-read; nt there: 256 MiB i1 / i2 / i4 decode 137 / 127 / 122 ->
  // 150 / 138 / 131 us), the apply pass reads nontemporally (132 / 127 / 120
  // us; tools/probe_dscan_nt.py, profiles/r02/probe_dscan_nt.json)
  const int ntm = mc_sched.dscan_nt;  // mc_sched.h
  if (ntm & 1) k_dscan_reduce_g<ES, true, BE><<<rg, MC_BLOCK, 0, st>>>(s, n, ws, ticket, ntiles, gt);
  else k_dscan_reduce_g<ES, false, BE><<<rg, MC_BLOCK, 0, st>>>(s, n, ws, ticket, ntiles, gt);
  if (ntm & 2) k_dscan_apply_g<ES, true, BE><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, ws, ntiles, gt);
  else k_dscan_apply_g<ES, false, BE><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, ws, ntiles, gt);
}

// mc_sched.dscan = 0 selects the generic three-pass kernels (lab A/B only)
static bool dscan_enabled() { return mc_sched.dscan != 0; }

template <int ES, bool BE = false>
static void launch_dscan(const uint8_t *s, uint8_t *d, size_t n, uint64_t *ws, hipStream_t st) {
  const size_t ntiles = (n + ds_tile<ES>() - 1) / ds_tile<ES>();
  const size_t ngroups = (ntiles + DS_GROUP - 1) / DS_GROUP;
  uint64_t *group = ws, *part = ws + ngroups, *gpre = part + DS_GROUP * ngroups;
  k_dscan_reduce<ES, BE><<<(unsigned)ngroups, MC_BLOCK, 0, st>>>(s, n, group, part);
  mc_launch_scan_sums_mw<false>(group, gpre, ngroups, st);
  k_dscan_apply<ES, BE><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, gpre, part);
}


// the speculative float path lives in mc_fspec.h, one translation unit per
// output dtype (mc_fspec_f2/f4/f8.hip: the walker instances dominate the
// build time)
static bool fspec_enabled() { return mc_sched.fspec != 0; }

static void launch_fspec_any(const uint8_t *s, uint8_t *d, size_t n, int a, int dt, void *ws, uint32_t *ticket,
                             hipStream_t st) {
  const bool swo = mc_dt_swapped(dt);
  dt = mc_dt_base(dt);
  if (swo || mc_dt_swapped(a)) {
    if (dt == MC_F8) mc_fspec_launch_be_f8(s, d, n, a, swo, ws, ticket, st);
    else if (dt == MC_F4) mc_fspec_launch_be_f4(s, d, n, a, swo, ws, ticket, st);
    else mc_fspec_launch_be_f2(s, d, n, a, swo, ws, ticket, st);
  } else if (dt == MC_F8) {
    mc_fspec_launch_f8(s, d, n, a, ws, ticket, st);
  } else if (dt == MC_F4) {
    mc_fspec_launch_f4(s, d, n, a, ws, ticket, st);
  } else {
    mc_fspec_launch_f2(s, d, n, a, ws, ticket, st);
  }
}

static void launch_fspec_rows_any(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a, int dt,
                                  uint64_t *fail, unsigned g, hipStream_t st) {
  const bool swo = mc_dt_swapped(dt);
  dt = mc_dt_base(dt);
  if (swo || mc_dt_swapped(a)) {
    if (dt == MC_F8) mc_fspec_rows_launch_be_f8(sc, ss, dc, ds, n, a, swo, fail, g, st);
    else if (dt == MC_F4) mc_fspec_rows_launch_be_f4(sc, ss, dc, ds, n, a, swo, fail, g, st);
    else mc_fspec_rows_launch_be_f2(sc, ss, dc, ds, n, a, swo, fail, g, st);
  } else if (dt == MC_F8) {
    mc_fspec_rows_launch_f8(sc, ss, dc, ds, n, a, fail, g, st);
  } else if (dt == MC_F4) {
    mc_fspec_rows_launch_f4(sc, ss, dc, ds, n, a, fail, g, st);
  } else {
    mc_fspec_rows_launch_f2(sc, ss, dc, ds, n, a, fail, g, st);
  }
}

// np.cumsum's first output is its first input cast to dtype; with the same
// float type up to byte order that cast moves bits, so a signalling NaN there
// keeps its payload.  The decode kernels compute element 0 through a value
// conversion (which quiets it) where the byte order changes or the type is
// f2: this one-thread-per-row pass re-writes it with the input's bits.
__global__ void k_first_elem_bits(const uint8_t *__restrict__ src, size_t ss, uint8_t *__restrict__ dst,
                                  size_t ds, size_t rows, int es, bool swap) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  uint64_t v = mc_load_elem_u(src + r * ss, 0, es);
  if (swap) v = mc_bswap_n(v, es);
  mc_store_elem_u(dst + r * ds, 0, es, v);
}

static void fix_first_elems(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t rows, int astype,
                            int dtype, hipStream_t st) {
  if (!mc_is_float(dtype) || mc_dt_base(astype) != mc_dt_base(dtype) || rows == 0) return;
  const bool swap = mc_dt_swapped(astype) != mc_dt_swapped(dtype);
  if (!swap && mc_dt_base(dtype) != MC_F2) return;
  k_first_elem_bits<<<(unsigned)((rows + 255) / 256), 256, 0, st>>>(s, ss, d, ds, rows, mc_itemsize(dtype), swap);
}

}  // namespace

int mc_delta_decode_batch_impl(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                               size_t nchunks, size_t n, int astype, int dtype, int variant,
                               mc_stream_t stream);

extern "C" {

size_t mc_delta_decode_workspace(size_t n, int astype, int dtype) {
  if (mc_ext_code(astype) || mc_ext_code(dtype)) return mc_ext_delta_decode_workspace(n, astype, dtype);
  if (mc_is_float(dtype)) return fspec_types_ok(astype, dtype) ? fspec_ws_bytes(n, dtype) : 0;
  const size_t generic = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE * sizeof(uint64_t);
  if (astype != dtype || dtype == MC_B1) return generic;
  const int es = mc_itemsize(dtype);
  const size_t three_pass = dscan_ws_entries(n, es) * sizeof(uint64_t);
  const size_t te = (size_t)(32 / es) * MC_BLOCK;
  const size_t two_launch = ((n + te - 1) / te + DS_MAX_GROUPS) * sizeof(uint32_t);  // tile + group totals
  size_t w = generic > three_pass ? generic : three_pass;
  return w > two_launch ? w : two_launch;
}

// np.cumsum(enc, out=dec) accumulates in promote_types(astype, dtype); the
// device reproduces that for a float dtype (any astype), an integer dtype
// from an integer/bool astype (wrap-around: the same modulo 2^bits) and
// bool from bool.  A float astype into an integer/bool dtype and an integer
// astype into bool are not implemented (MC_EINVAL, never different bytes).
static bool delta_decode_pair_ok(int astype, int dtype) {
  if (mc_is_float(dtype)) return true;
  if (mc_is_float(astype)) return false;
  return dtype != MC_B1 || astype == MC_B1;
}

int mc_delta_decode(const void *src, void *dst, size_t n, int astype, int dtype, void *workspace,
                    size_t workspace_bytes, uint32_t *ticket, mc_stream_t stream) {
  if (ticket && (uintptr_t)ticket % 8) return MC_EINVAL;
  if (mc_ext_code(astype) || mc_ext_code(dtype))
    return mc_ext_delta_decode(src, dst, n, astype, dtype, workspace, workspace_bytes, ticket, (hipStream_t)stream);
  if (!mc_valid_dtype(dtype) || !mc_valid_dtype(astype)) return MC_EINVAL;
  if (!delta_decode_pair_ok(astype, dtype)) return MC_EINVAL;
  if (n == 0) return MC_OK;
  if (!src || !dst) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  if (mc_is_float(dtype)) {
    // speculative parallel scan + verification, serial fix-up (above); the
    // plain serial chain where the preconditions (workspace, alignment,
    // astype == dtype, f4/f8) do not hold
    if (fspec_types_ok(astype, dtype) && fspec_enabled() && workspace &&
        workspace_bytes >= fspec_ws_bytes(n, dtype) && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0 &&
        (uintptr_t)workspace % 8 == 0) {
      launch_fspec_any(s, d, n, astype, dtype, workspace, ticket, st);
      fix_first_elems(s, 0, d, 0, 1, astype, dtype, st);
      return mc_last_launch();
    }
    mc_launch_serial_any(s, 0, d, 0, n, 1, astype, dtype, st);
    fix_first_elems(s, 0, d, 0, 1, astype, dtype, st);
    return mc_last_launch();
  }
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  if (!workspace || workspace_bytes < mc_delta_decode_workspace(n, astype, dtype)) return MC_ENOSPC;
  uint64_t *sums = static_cast<uint64_t *>(workspace);
  if (astype == dtype && dtype != MC_B1 && ((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 16) == 0 &&
      dscan_enabled()) {
    const int es = mc_itemsize(dtype);
    const bool be = mc_dt_swapped(dtype);  // both big-endian: reversed in registers
    // two launches with a ticket while groups stay <= 1024 tiles (the apply
    // workgroup sums its group's earlier tile totals, 4 per thread)
    if (ticket && es <= 4 && ds_group_tiles((n + (size_t)(32 / es) * MC_BLOCK - 1) / ((size_t)(32 / es) * MC_BLOCK)) <= 1024) {
      uint32_t *ws = static_cast<uint32_t *>(workspace);
      if (es == 1) launch_dscan_g<1>(s, d, n, ws, ticket, st);
      else if (es == 2) be ? launch_dscan_g<2, true>(s, d, n, ws, ticket, st) : launch_dscan_g<2>(s, d, n, ws, ticket, st);
      else be ? launch_dscan_g<4, true>(s, d, n, ws, ticket, st) : launch_dscan_g<4>(s, d, n, ws, ticket, st);
      return mc_last_launch();
    }
    switch (es) {
      case 1: launch_dscan<1>(s, d, n, sums, st); break;
      case 2: be ? launch_dscan<2, true>(s, d, n, sums, st) : launch_dscan<2>(s, d, n, sums, st); break;
      case 4: be ? launch_dscan<4, true>(s, d, n, sums, st) : launch_dscan<4>(s, d, n, sums, st); break;
      default: be ? launch_dscan<8, true>(s, d, n, sums, st) : launch_dscan<8>(s, d, n, sums, st); break;
    }
    return mc_last_launch();
  }
  const bool vec = ((uintptr_t)src % (4 * mc_itemsize(astype)) == 0) &&
                   ((uintptr_t)dst % (4 * mc_itemsize(dtype)) == 0);
  if (dtype == MC_B1) {
    if (vec) launch_int_scan<true, -1, -1, true>(s, d, n, astype, dtype, sums, ntiles, st);
    else launch_int_scan<true, -1, -1, false>(s, d, n, astype, dtype, sums, ntiles, st);
  } else if (vec && astype == MC_I2 && dtype == MC_I2) {
    launch_int_scan<false, MC_I2, MC_I2, true>(s, d, n, astype, dtype, sums, ntiles, st);
  } else if (vec && astype == MC_I4 && dtype == MC_I4) {
    launch_int_scan<false, MC_I4, MC_I4, true>(s, d, n, astype, dtype, sums, ntiles, st);
  } else if (vec) {
    launch_int_scan<false, -1, -1, true>(s, d, n, astype, dtype, sums, ntiles, st);
  } else {
    launch_int_scan<false, -1, -1, false>(s, d, n, astype, dtype, sums, ntiles, st);
  }
  return mc_last_launch();
}

int mc_delta_decode_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                          size_t nchunks, size_t n, int astype, int dtype, mc_stream_t stream) {
  return mc_delta_decode_batch_impl(src, src_stride, dst, dst_stride, nchunks, n, astype, dtype, 0,
                                    stream);
}

size_t mc_delta_decode_batch_workspace(size_t nchunks, size_t n, int astype, int dtype) {
  (void)n;
  return fspec_types_ok(astype, dtype) ? nchunks * sizeof(uint64_t) : 0;
}

int mc_delta_decode_batch_ws(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                             size_t nchunks, size_t n, int astype, int dtype, void *workspace,
                             size_t workspace_bytes, mc_stream_t stream) {
  const bool spec = fspec_types_ok(astype, dtype) && fspec_enabled() && workspace &&
                    workspace_bytes >= nchunks * sizeof(uint64_t) && (uintptr_t)workspace % 8 == 0 &&
                    (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0 &&
                    (nchunks == 1 || (src_stride % 16 == 0 && dst_stride % 16 == 0));
  if (!spec || n == 0 || nchunks == 0 || !src || !dst ||
      (nchunks > 1 && (src_stride < n * mc_itemsize(astype) || dst_stride < n * mc_itemsize(dtype))))
    return mc_delta_decode_batch(src, src_stride, dst, dst_stride, nchunks, n, astype, dtype, stream);
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint64_t *fail = static_cast<uint64_t *>(workspace);
  constexpr size_t GRID_MAX = 1u << 30;
  for (size_t c0 = 0; c0 < nchunks; c0 += GRID_MAX) {
    const unsigned g = (unsigned)min(GRID_MAX, nchunks - c0);
    const uint8_t *sc = s + c0 * src_stride;
    uint8_t *dc = d + c0 * dst_stride;
    launch_fspec_rows_any(sc, src_stride, dc, dst_stride, n, astype, dtype, fail + c0, g, st);
    fix_first_elems(sc, src_stride, dc, dst_stride, g, astype, dtype, st);
  }
  return mc_last_launch();
}

}  // extern "C"

// Batched Delta decode with an explicit float-chain schedule (0 = default by
// batch size; 1-5 the LDS slot / read-group sweep of tools/lab).  C++
// linkage: the C ABI exposes the default only (mc_delta_decode_batch).
int mc_delta_decode_batch_impl(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                               size_t nchunks, size_t n, int astype, int dtype, int variant,
                               mc_stream_t stream) {
  if (variant < 0 || variant > 5) return MC_EINVAL;
  if (!mc_valid_dtype(dtype) || !mc_valid_dtype(astype)) return MC_EINVAL;
  if (!delta_decode_pair_ok(astype, dtype)) return MC_EINVAL;
  if (n == 0 || nchunks == 0) return MC_OK;
  if (!src || !dst) return MC_EINVAL;
  if (nchunks > 1 && (src_stride < n * mc_itemsize(astype) || dst_stride < n * mc_itemsize(dtype)))
    return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  constexpr size_t GRID_MAX = 1u << 30;
  for (size_t c0 = 0; c0 < nchunks; c0 += GRID_MAX) {
    const size_t rows = min(GRID_MAX, nchunks - c0);
    const uint8_t *sc = s + c0 * src_stride;
    uint8_t *dc = d + c0 * dst_stride;
    if (mc_is_float(dtype)) {
      mc_launch_serial_any(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st, variant);
      fix_first_elems(sc, src_stride, dc, dst_stride, rows, astype, dtype, st);
      continue;
    }
    const size_t as = mc_itemsize(astype), ds = mc_itemsize(dtype);
    const bool vec = ((uintptr_t)sc % (4 * as) == 0) && (src_stride % (4 * as) == 0) &&
                     ((uintptr_t)dc % (4 * ds) == 0) && (dst_stride % (4 * ds) == 0);
    const bool al16 = ((uintptr_t)sc % 16 == 0) && (rows == 1 || src_stride % 16 == 0) &&
                      ((uintptr_t)dc % 16 == 0) && (rows == 1 || dst_stride % 16 == 0);
    if (astype == dtype && dtype != MC_B1 && al16 && dscan_enabled()) {
      const unsigned g = (unsigned)rows;
      const bool be = mc_dt_swapped(dtype);
      switch (ds) {
        case 1: k_dscan_rows<1><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n); break;
        case 2:
          if (be) k_dscan_rows<2, true><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n);
          else k_dscan_rows<2><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n);
          break;
        case 4:
          if (be) k_dscan_rows<4, true><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n);
          else k_dscan_rows<4><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n);
          break;
        default:
          if (be) k_dscan_rows<8, true><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n);
          else k_dscan_rows<8><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n);
          break;
      }
      continue;
    }
    if (dtype == MC_B1) {
      if (vec) launch_rows<true, -1, -1, true>(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st);
      else launch_rows<true, -1, -1, false>(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st);
    } else if (vec && astype == MC_I2 && dtype == MC_I2) {
      launch_rows<false, MC_I2, MC_I2, true>(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st);
    } else if (vec && astype == MC_I4 && dtype == MC_I4) {
      launch_rows<false, MC_I4, MC_I4, true>(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st);
    } else if (vec) {
      launch_rows<false, -1, -1, true>(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st);
    } else {
      launch_rows<false, -1, -1, false>(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st);
    }
  }
  return mc_last_launch();
}
