// mc_fspec.h -- the speculative float Delta decode (delta.py:69-83,
// np.cumsum(enc, out=dec) for float dtypes): templates shared by the
// per-dtype translation units mc_fspec_f2.hip, mc_fspec_f4.hip and
// mc_fspec_f8.hip (one output dtype each, so the instances build in
// parallel).  The entry points in mc_scan.hip dispatch to them.
#pragma once

#include "mc_scan.h"

namespace {

// ---------------------------------------------------------------------------
// Speculative float Delta decode (one chunk, astype == dtype in {f4, f8}).
// numpy's cumsum rounds after every add, so in general the adds form one
// serial chain.  But when every add happens to be exact -- the common case
// for the output of a Delta encode of slowly varying values, where each
// difference is exact (Sterbenz) and adding it back is exact too -- the
// serial result IS the exact prefix sum, which a parallel scan computes.
// So the decode speculates and verifies:
//   1. k_fspec_reduce: per-tile total of the tile's prefix sums in double,
//      with the same block-scan code as the apply pass, so a tile's total is
//      bitwise the value its last element's candidate is built from;
//   2. k_fspec_pre: exclusive scan of the totals (any order: each tile only
//      uses its own prefix and its predecessor's) and reset of the
//      first-failure word;
//   3. k_fspec_apply: candidate c_i = dtype(S_tile + local prefix_i); every
//      element checks c_i == dtype(c_{i-1} + enc_i) bitwise -- numpy's
//      recurrence itself -- with non-finite values counted as failures, and
//      the smallest failing index goes to one word (atomicMin; tiles past a
//      recorded failure skip their work);
//   4. k_scan_serial in fix-up mode reruns the serial chain from that index
//      with the verified value before it (returns at once when nothing
//      failed).
// The candidates are a deterministic function of the input, so the first
// failure is always recorded, and by induction from c_0 = enc_0 every
// element before it equals numpy's serial value; after it the chain is
// serial again.  The output is bit-exact for any input; the data only decide
// how much of the chunk runs at scan speed instead of one add per element.
// ---------------------------------------------------------------------------
// A thread holds FS_Q 16-B vectors of OUTPUT elements (W = 16 / itemsize(D)
// each) in FS_Q segments of the tile: segment q is W*MC_BLOCK contiguous
// elements and thread t owns its vector at W*t, so every wave store covers
// 1 KiB contiguously; 16 KiB of output per tile (8192 f2 / 4096 f4 / 2048 f8
// elements).
//
// FsT<A_, D> is the element model, numpy's cumsum(enc, out=dec) with enc of
// dtype A (astype) and dec of dtype D (a float dtype), exactly as the serial
// chain runs it (k_scan_serial): every input is first cast to D
// (mc_num_cast), the adds happen in D -- f2 as float32 adds rounded to half
// per step (ser_add<MC_F2>) -- and c_0 = D(enc_0).  A_ = D loads 16-B
// vectors of D; A_ = -1 (any other astype, given at run time) loads element
// by element and casts.  The double-precision scan only proposes candidates;
// the per-element check against that recurrence decides, so the candidate
// rounding (double -> D) need not match numpy's.
// P: the precision of the candidate scan (double; float for f2, whose
// 11-bit values sum exactly in float32 over a tile of smooth data and whose
// double scan made the f2 instances VALU-bound -- any precision only
// proposes, the per-element check decides)
template <int D> struct FsStore { using S = float; using V = float; using P = double; };
template <> struct FsStore<MC_F8> { using S = double; using V = double; using P = double; };
template <> struct FsStore<MC_F2> { using S = _Float16; using V = float; using P = float; };

template <int A_, int D>
struct FsT {
  using S = typename FsStore<D>::S;  // stored element
  using V = typename FsStore<D>::V;  // arithmetic value (numpy's loop type)
  using P = typename FsStore<D>::P;  // candidate scan precision
  static constexpr int W = 16 / (int)sizeof(S);
  typedef S svec __attribute__((ext_vector_type(W)));
  MC_DEV static V from_bits(uint64_t bits, int a) {  // enc element -> its D value
    return (V)mc_num_cast(mc_num_from_bits(bits, a), a, D).f;
  }
  MC_DEV static S round(P x) { return (S)x; }  // candidate (any rounding)
  // the last candidate of a tile from its (double) tile prefix and total, as
  // the apply pass / walker computed it there (bitwise)
  MC_DEV static S bound(double pre, double sum) { return round((P)pre + (P)sum); }
  MC_DEV static V val(S c) { return (V)c; }
  MC_DEV static S store(V r) { return (S)r; }  // exact: r holds a D value
  MC_DEV static V step(V pv, V x) { return ser_add<D>(pv, x); }
  MC_DEV static uint64_t bits(S c) {
    if constexpr (sizeof(S) == 8) return __builtin_bit_cast(uint64_t, c);
    else if constexpr (sizeof(S) == 4) return __builtin_bit_cast(uint32_t, c);
    else return __builtin_bit_cast(uint16_t, c);
  }
  MC_DEV static bool finite(S c) {
    if constexpr (sizeof(S) == 8) return __builtin_isfinite(c);
    else return __builtin_isfinite((float)c);
  }
  // the candidate of lane - 1 (lane 0 keeps its own, as __shfl_up(c, 1)
  // would): the bit pattern moved by DPP wave_shr:1, no LDS round trip
  MC_DEV static S shfl_up1(S c) {
    if constexpr (sizeof(S) == 8) {
      const uint64_t b = __builtin_bit_cast(uint64_t, c);
      const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
      return __builtin_bit_cast(S, ((uint64_t)mc_wave_shr1(hi, hi) << 32) | mc_wave_shr1(lo, lo));
    } else if constexpr (sizeof(S) == 4) {
      const uint32_t b = __builtin_bit_cast(uint32_t, c);
      return __builtin_bit_cast(S, mc_wave_shr1(b, b));
    } else {
      const uint32_t b = __builtin_bit_cast(uint16_t, c);
      return __builtin_bit_cast(S, (uint16_t)mc_wave_shr1(b, b));
    }
  }
};

// Byte order (SW, bit 0: the input is big-endian, bit 1: the output is): a
// constant-astype instance (A_ >= 0) reverses each element's bytes after its
// vector load; a runtime astype (A_ = -1) arrives as a flagged code and its
// loads go through mc_num_from_bits; a big-endian output is reversed before
// every store.  The whole 16-B vector is bit-cast, never one component (a
// component bit cast reads component 0 on gfx950).
template <typename V>
MC_DEV V fs_bswap(V x) {
  static_assert(sizeof(V) == 16, "16-B vectors");
  return __builtin_bit_cast(V, mc_bswap_vec<(int)sizeof(x[0])>(__builtin_bit_cast(mc_u32x4, x)));
}
template <typename S>
MC_DEV S fs_bswap_scalar(S c) {
  if constexpr (sizeof(S) == 8) return __builtin_bit_cast(S, __builtin_bswap64(__builtin_bit_cast(uint64_t, c)));
  else if constexpr (sizeof(S) == 4) return __builtin_bit_cast(S, __builtin_bswap32(__builtin_bit_cast(uint32_t, c)));
  else return __builtin_bit_cast(S, __builtin_bswap16(__builtin_bit_cast(uint16_t, c)));
}

template <int D> constexpr size_t fs_tile() { return fs_tile_of(D); }

template <int D>
MC_DEV size_t fs_elem0(size_t t0, int q) {  // first element of this thread's vector in segment q
  return t0 + (size_t)q * fs_w_of(D) * MC_BLOCK + (size_t)threadIdx.x * fs_w_of(D);
}

template <int A_, int D, int SW = 0>
MC_DEV void fs_load(const uint8_t *src, size_t n, size_t t0, int a,
                    typename FsT<A_, D>::V (&v)[FS_Q][FsT<A_, D>::W]) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
  if constexpr (A_ == D) {
    // default-policy loads: the apply pass re-reads what the reduce pass read
    // and finds part of it in the Infinity Cache (256 MiB f4 smooth decode
    // 158-162 -> 154 us against nontemporal loads; f8 unchanged)
    // every load first, then the byte swaps / conversions: a swap between
    // the (bounds-branched) loads waited for each load before the next issued
    typename Tr::svec xs[FS_Q];
    if (t0 + fs_tile<D>() <= n) {
      // a whole tile in range (every tile but a chunk's last): the FS_Q
      // vector loads with no branch between them, so they are all in flight
      // together (bounds-branched, each load was waited for before the next
      // issued -- four round trips per workgroup, round 5)
#pragma unroll
      for (int q = 0; q < FS_Q; ++q)
        xs[q] = *reinterpret_cast<const typename Tr::svec *>(src + fs_elem0<D>(t0, q) * sizeof(typename Tr::S));
    } else {
#pragma unroll
      for (int q = 0; q < FS_Q; ++q) {
        const size_t e0 = fs_elem0<D>(t0, q);
        if (e0 + W <= n) {
          xs[q] = *reinterpret_cast<const typename Tr::svec *>(src + e0 * sizeof(typename Tr::S));
        } else {
#pragma unroll
          for (int e = 0; e < W; ++e)
            xs[q][e] = e0 + e < n ? reinterpret_cast<const typename Tr::S *>(src)[e0 + e] : (typename Tr::S)0;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
      typename Tr::svec x = xs[q];
      if constexpr ((SW & 1) != 0) x = fs_bswap(x);
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = (typename Tr::V)x[e];
    }
  } else if constexpr (A_ == MC_F4 && D == MC_F8) {
    static_assert((SW & 1) == 0, "big-endian f4 input takes the runtime-astype instance");
    // f8 <- f4 (the dispatch checks 8-B alignment): one 8-B load of the
    // thread's 2 float32 per vector, the casts in registers.  The components
    // are copied out before the bit casts: __builtin_bit_cast of an
    // ext_vector component reads component 0 (seen in the gfx950 assembly)
    if (t0 + fs_tile<D>() <= n) {  // a whole tile: every load in flight together (see above)
      mc_u32x2 xs[FS_Q];
#pragma unroll
      for (int q = 0; q < FS_Q; ++q) xs[q] = mc_ld8<false>(src + fs_elem0<D>(t0, q) * 4);
#pragma unroll
      for (int q = 0; q < FS_Q; ++q) {
        const uint32_t x0 = xs[q].x, x1 = xs[q].y;
        v[q][0] = (double)__builtin_bit_cast(float, x0);
        v[q][1] = (double)__builtin_bit_cast(float, x1);
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
      const size_t e0 = fs_elem0<D>(t0, q);
      if (e0 + W <= n) {
        const mc_u32x2 x = mc_ld8<false>(src + e0 * 4);
        const uint32_t x0 = x.x, x1 = x.y;
        v[q][0] = (double)__builtin_bit_cast(float, x0);
        v[q][1] = (double)__builtin_bit_cast(float, x1);
      } else {
#pragma unroll
        for (int e = 0; e < W; ++e)
          v[q][e] = e0 + e < n ? (double)reinterpret_cast<const float *>(src)[e0 + e] : 0.0;
      }
    }
  } else {
    const int as = mc_itemsize(a);
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
      const size_t e0 = fs_elem0<D>(t0, q);
      uint64_t b[W];
#pragma unroll
      for (int e = 0; e < W; ++e) b[e] = e0 + e < n ? mc_load_elem_u(src, e0 + e, as) : 0;
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = e0 + e < n ? Tr::from_bits(b[e], a) : (typename Tr::V)0;
    }
  }
}

template <int A_, int D, int SW = 0>
MC_DEV void fs_store(uint8_t *dst, size_t n, size_t t0, const typename FsT<A_, D>::S (&c)[FS_Q][FsT<A_, D>::W]) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    const size_t e0 = fs_elem0<D>(t0, q);
    if (e0 + W <= n) {
      typename Tr::svec x;
#pragma unroll
      for (int e = 0; e < W; ++e) x[e] = c[q][e];
      if constexpr ((SW & 2) != 0) x = fs_bswap(x);
      __builtin_nontemporal_store(x, reinterpret_cast<typename Tr::svec *>(dst + e0 * sizeof(typename Tr::S)));
    } else {
      for (int e = 0; e < W && e0 + e < n; ++e)
        reinterpret_cast<typename Tr::S *>(dst)[e0 + e] = (SW & 2) ? fs_bswap_scalar(c[q][e]) : c[q][e];
    }
  }
}

// p[q][e] = the tile-relative inclusive prefix sum (double) of this thread's
// element e of segment q.  Fixed association (element, lane, wave, segment
// order), so the reduce and apply passes compute bitwise the same values.
// Wave-wide inclusive scan of one double per lane by DPP moves (row_shr 1, 2,
// 4, 8 inside each row of 16 lanes, then row_bcast 15 / 31 across rows):
// 12 v_mov_dpp + 6 adds, no LDS (the __shfl_up Hillis-Steele scan is 12
// ds_bpermute round trips).  Lanes without a source add -0.0, the exact
// identity (x + -0.0 == x bitwise for every x but a signalling NaN, and the
// speculative scan treats non-finite values as failures anyway).
template <int CTRL, int ROW_MASK>
MC_DEV double mc_dpp_f64(double x) {
  const uint64_t xb = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)xb, CTRL, ROW_MASK, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)0x80000000u, (int)(uint32_t)(xb >> 32), CTRL,
                                                            ROW_MASK, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
MC_DEV double mc_wave_scan_f64(double x) {
  x = x + mc_dpp_f64<0x111, 0xF>(x);  // row_shr:1
  x = x + mc_dpp_f64<0x112, 0xF>(x);  // row_shr:2
  x = x + mc_dpp_f64<0x114, 0xF>(x);  // row_shr:4
  x = x + mc_dpp_f64<0x118, 0xF>(x);  // row_shr:8
  x = x + mc_dpp_f64<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3
  x = x + mc_dpp_f64<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
// lane i <- lane i - 1 (lane 0 <- -0.0)
MC_DEV double mc_wave_shr1_f64(double x) { return mc_dpp_f64<0x138, 0xF>(x); }

// the same for one float per lane (6 DPP-sourced adds)
template <int CTRL, int ROW_MASK>
MC_DEV float mc_dpp_f32(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp((int)0x80000000u, __builtin_bit_cast(int, x), CTRL,
                                                               ROW_MASK, 0xF, false));
}
MC_DEV float mc_wave_scan_f32(float x) {
  x = x + mc_dpp_f32<0x111, 0xF>(x);
  x = x + mc_dpp_f32<0x112, 0xF>(x);
  x = x + mc_dpp_f32<0x114, 0xF>(x);
  x = x + mc_dpp_f32<0x118, 0xF>(x);
  x = x + mc_dpp_f32<0x142, 0xA>(x);
  x = x + mc_dpp_f32<0x143, 0xC>(x);
  return x;
}
MC_DEV float mc_wave_shr1_f32(float x) { return mc_dpp_f32<0x138, 0xF>(x); }
MC_DEV double mc_wave_scan_p(double x) { return mc_wave_scan_f64(x); }
MC_DEV float mc_wave_scan_p(float x) { return mc_wave_scan_f32(x); }
MC_DEV double mc_wave_shr1_p(double x) { return mc_wave_shr1_f64(x); }
MC_DEV float mc_wave_shr1_p(float x) { return mc_wave_shr1_f32(x); }

template <typename V, int W, typename P>
MC_DEV void fs_tile_scan(const V (&v)[FS_Q][W], P (&p)[FS_Q][W], P (&lds)[FS_Q][MC_BLOCK / 64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  P incl[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    p[q][0] = (P)v[q][0];
#pragma unroll
    for (int e = 1; e < W; ++e) p[q][e] = p[q][e - 1] + (P)v[q][e];
    incl[q] = p[q][W - 1];
  }
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) incl[q] = mc_wave_scan_p(incl[q]);
  P ex[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    if (lane == 63) lds[q][wave] = incl[q];
    ex[q] = mc_wave_shr1_p(incl[q]);
  }
  __syncthreads();
  P base = 0;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    P w = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < MC_BLOCK / 64; ++j) {
      if (j < wave) w = w + lds[q][j];
      tot = tot + lds[q][j];
    }
    const P pre = base + (lane ? w + ex[q] : w);
#pragma unroll
    for (int e = 0; e < W; ++e) p[q][e] = pre + p[q][e];
    base = base + tot;
  }
}

// The smallest global index in this thread's FS_Q x W candidates c whose
// value differs (bitwise) from numpy's recurrence D(pred + x), or that is
// not finite; ~0 if none.  p0[q] = the predecessor candidate of the
// thread's first element of segment q.
template <int A_, int D>
MC_DEV uint64_t fs_check(const typename FsT<A_, D>::S (&c)[FS_Q][FsT<A_, D>::W],
                         const typename FsT<A_, D>::V (&v)[FS_Q][FsT<A_, D>::W],
                         const typename FsT<A_, D>::S (&p0)[FS_Q], size_t t0, size_t n) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
  uint64_t first = ~(uint64_t)0;
#pragma unroll
  for (int q = FS_Q - 1; q >= 0; --q) {  // descending: the last hit is the smallest index
    const size_t e0 = fs_elem0<D>(t0, q);
#pragma unroll
    for (int e = W - 1; e >= 0; --e) {
      const size_t g = e0 + e;
      const typename Tr::S pv = e ? c[q][e - 1] : p0[q];
      const typename Tr::S r = g == 0 ? Tr::store(v[q][0]) : Tr::store(Tr::step(Tr::val(pv), v[q][e]));
      // a non-finite input makes its own prefix (and so c) non-finite
      const bool ok = Tr::bits(c[q][e]) == Tr::bits(r) && Tr::finite(c[q][e]);
      if (g < n && !ok) first = g;
    }
  }
  return first;
}

// the wave's smallest failing index (~0 if none): one ballot when no lane
// failed (the common case of smooth data), the min-reduction otherwise
MC_DEV uint64_t fs_wave_min_fail(uint64_t first) {
  if (__builtin_amdgcn_ballot_w64(first != ~(uint64_t)0) == 0) return ~(uint64_t)0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(first, off, 64);
    first = o < first ? o : first;
  }
  return first;
}

template <int A_, int D, int SW = 0>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_reduce(const uint8_t *__restrict__ src, size_t n, int a,
                                                          double *__restrict__ sums) {
  using Tr = FsT<A_, D>;
  using P = typename Tr::P;
  constexpr int W = Tr::W;
  __shared__ P lds[FS_Q][MC_BLOCK / 64];
  typename Tr::V v[FS_Q][W];
  fs_load<A_, D, SW>(src, n, (size_t)blockIdx.x * fs_tile<D>(), a, v);
  P p[FS_Q][W];
  fs_tile_scan<typename Tr::V, W, P>(v, p, lds);
  if (threadIdx.x == MC_BLOCK - 1) sums[blockIdx.x] = (double)p[FS_Q - 1][W - 1];
}

// VERDICT r5 item 2 asked for k_fspec_pre's launch to be folded away, as the
// integer scans fold theirs.  Four forms were built and measured against
// this one on one box (256 MiB f4 of smooth data, the whole decode through
// mc_delta_decode with and without a ticket, 7 interleaved rounds of 20
// calls, tools/probe_fspec_fold.py, profiles/r06/probe_fspec_fold_*.json):
//   * the reduce pass's last arrivers scan the tile totals (group words in
//     the arrival ticket, sc1 hand-offs): 130.3 against 129.1 us -- every
//     workgroup waits for its returning arrival, the reduce pass 44 -> 52.5;
//   * the apply pass rebuilds its prefix from group accumulators (no-return
//     float atomics in the ticket) and the earlier totals of its group:
//     138.2 against 127.4 us -- two more dependent round trips per apply
//     workgroup, the apply pass 78 -> 95.6;
//   * k_fspec_pre over group accumulators (one workgroup per group, ~2 loads
//     per thread: 4.8 instead of 6.5 us): 129.1 against 128.2 us -- the
//     reduce pass's float atomics cost more (44 -> 49.6), also with the tiles
//     permuted over the groups (50.5; 131.9 against 130.2).
// None wins, so the decode keeps reduce -> k_fspec_pre -> apply -> walk.
template <int A_, int D, int SW = 0>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_apply(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t n, int a,
                                                         const double *__restrict__ sums,
                                                         const double *__restrict__ pre_t,
                                                         uint64_t *__restrict__ tfail,
                                                         uint64_t *__restrict__ fail) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  using P = typename Tr::P;
  constexpr int W = Tr::W;
  __shared__ P lds[FS_Q][MC_BLOCK / 64];
  __shared__ S ldsc[FS_Q][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t tile = blockIdx.x;
  const size_t t0 = tile * fs_tile<D>();
  // every tile is verified and stored, also past an earlier failure: the
  // walker (k_fspec_walk) re-bases at the first failing element and jumps
  // over the tiles recorded here as verified once it is back in sync
  typename Tr::V v[FS_Q][W];
  fs_load<A_, D, SW>(src, n, t0, a, v);
  P p[FS_Q][W];
  fs_tile_scan<typename Tr::V, W, P>(v, p, lds);
  const P Sp = (P)pre_t[tile];  // the tile's prefix
  S c[FS_Q][W], up[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
#pragma unroll
    for (int e = 0; e < W; ++e) c[q][e] = Tr::round(Sp + p[q][e]);
    up[q] = Tr::shfl_up1(c[q][W - 1]);
    if (lane == 63) ldsc[q][wave] = c[q][W - 1];
  }
  __syncthreads();
  // the tile's last candidate in the previous tile: the same double sum it
  // was rounded from there (sums[] is that tile's last prefix, bitwise)
  const S pbound = tile ? Tr::bound(pre_t[tile - 1], sums[tile - 1]) : (S)0;
  S p0[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    if (lane) p0[q] = up[q];
    else if (wave) p0[q] = ldsc[q][wave - 1];
    else p0[q] = q ? ldsc[q - 1][MC_BLOCK / 64 - 1] : pbound;
  }
  uint64_t first = fs_check<A_, D>(c, v, p0, t0, n);
  fs_store<A_, D, SW>(dst, n, t0, c);
  first = fs_wave_min_fail(first);
  if (lane == 0 && first != ~(uint64_t)0) {
    atomicMin((unsigned long long *)(tfail + tile), (unsigned long long)first);
    atomicMin((unsigned long long *)fail, (unsigned long long)first);
  }
}

// Batched speculative float Delta decode: one workgroup per chunk walks it
// in tiles with a running double prefix `carry` (the next tile's candidates
// are carry + in-tile prefix, and its first element's predecessor is the
// previous tile's last candidate), verifying every element as in
// k_fspec_apply.  At the first tile with a failing element the workgroup
// records the tile's start in fail[row] and stops without storing it; the
// walker (k_fspec_walk, one workgroup per row) resumes that row there.
// fail[row] = n when the whole row verified.
template <int A_, int D, int SW = 0>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_rows(const uint8_t *__restrict__ src,
                                                        size_t src_stride, uint8_t *__restrict__ dst,
                                                        size_t dst_stride, size_t n, int a,
                                                        uint64_t *__restrict__ fail) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  using P = typename Tr::P;
  constexpr int W = Tr::W;
  __shared__ P lds[2][FS_Q][MC_BLOCK / 64];
  __shared__ S ldsc[2][FS_Q][MC_BLOCK / 64];
  __shared__ uint64_t ldsf[2][MC_BLOCK / 64];
  __shared__ P ldsp[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  src += (size_t)blockIdx.x * src_stride;
  dst += (size_t)blockIdx.x * dst_stride;
  P carry = 0;
  S prevc = (S)0;
  int par = 0;
  typename Tr::V nv[FS_Q][W];
  fs_load<A_, D, SW>(src, n, 0, a, nv);
  for (size_t t0 = 0; t0 < n; t0 += fs_tile<D>(), par ^= 1) {
    typename Tr::V v[FS_Q][W];
#pragma unroll
    for (int q = 0; q < FS_Q; ++q)
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = nv[q][e];
    if (t0 + fs_tile<D>() < n) fs_load<A_, D, SW>(src, n, t0 + fs_tile<D>(), a, nv);  // next tile in flight
    P p[FS_Q][W];
    fs_tile_scan<typename Tr::V, W, P>(v, p, lds[par]);
    S c[FS_Q][W], up[FS_Q];
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
#pragma unroll
      for (int e = 0; e < W; ++e) c[q][e] = Tr::round(carry + p[q][e]);
      up[q] = Tr::shfl_up1(c[q][W - 1]);
      if (lane == 63) ldsc[par][q][wave] = c[q][W - 1];
    }
    __syncthreads();
    S p0[FS_Q];
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
      if (lane) p0[q] = up[q];
      else if (wave) p0[q] = ldsc[par][q][wave - 1];
      else p0[q] = q ? ldsc[par][q - 1][MC_BLOCK / 64 - 1] : prevc;
    }
    const uint64_t first = fs_wave_min_fail(fs_check<A_, D>(c, v, p0, t0, n));
    if (lane == 0) ldsf[par][wave] = first;
    if (threadIdx.x == MC_BLOCK - 1) ldsp[par] = carry + p[FS_Q - 1][W - 1];
    __syncthreads();
    uint64_t tf = ldsf[par][0];
#pragma unroll
    for (int j = 1; j < MC_BLOCK / 64; ++j) tf = ldsf[par][j] < tf ? ldsf[par][j] : tf;
    if (tf != ~(uint64_t)0) {  // uniform across the workgroup
      // the failing tile is not stored: the serial fix-up restarts at its
      // first element (a chunk that fails in its first tile -- random data --
      // then costs the serial chain alone, with no speculative stores)
      if (threadIdx.x == 0) fail[blockIdx.x] = t0;
      return;
    }
    fs_store<A_, D, SW>(dst, n, t0, c);
    // next tile: prefix = this tile's last prefix (thread MC_BLOCK-1's, via
    // LDS), predecessor = this tile's last candidate
    carry = ldsp[par];
    prevc = ldsc[par][FS_Q - 1][MC_BLOCK / 64 - 1];
  }
  if (threadIdx.x == 0) fail[blockIdx.x] = n;
}

// ---------------------------------------------------------------------------
// The walker: re-speculation after a failure, one workgroup per chunk.
//
// A failing element f means the candidates after f carry the wrong running
// error: numpy's chain rounded at or before f, so its values are no longer
// the exact prefix sums.  The chain's state is one value, and from a TRUE
// value y_f the same speculation works again: candidates
// c_i = D(y_f + (p_i - p_f)) (p = the tile's double prefix) verified per
// element exactly as above.  The walker visits a chunk's tiles in order,
// carrying the true value at each tile boundary, and inside a tile re-bases
// at every failing element: the smallest failing index f is fixed with one
// add of numpy's recurrence (c_{f-1} is verified), the candidates after it
// are recomputed from y_f, and the tile is verified again -- so the serial
// work is one add per rounding event, not one add per element.  Measured on
// f4 data with rounding events (tools/fspec_model.py): 2-20 re-basings per
// 4096-element tile for noisy sines, random walks, chirps and sparse data.
// A tile that needs more than FSW_CAP re-basings (noise-like data, ~500 per
// tile) finishes as a serial chain over its values staged in LDS, and the
// following tiles start serial too, trying speculation again every
// FSW_PROBE tiles.  By induction every tile starts from the true value, so
// the output is bit-exact for any input.
//
// Single chunk: after k_fspec_apply (which verifies every tile against the
// global prefix and records each tile's first failing index) one walker
// starts at the first failing tile.  Whenever a tile ends on the value the
// apply pass used as the next tile's predecessor, the walker is "in sync"
// again: the following tiles that verified at apply time are already correct
// in dst, so it jumps to the next tile that failed there.
// Batches (one walker per chunk): every tile is walked, carrying the true
// value; rowfail[row] = the first index that needed a re-basing (n if none).
// ---------------------------------------------------------------------------
constexpr int FSW_CAP = 16;        // re-basings per tile before the serial fallback
constexpr int FSW_PROBE = 8;       // after a serial tile, the FSW_PROBE-th tile on speculates again ...
constexpr int FSW_PROBE_CAP = 2;   // ... with at most this many re-basings; each failed probe doubles
constexpr int FSW_PROBE_MAX = 64;  // the gap up to this (noise costs ~0.5 % over the plain chain)
constexpr int FSW_G = 32;          // serial chain: values per LDS read group (8 x 16 B in flight)
constexpr int FSW_NW = MC_BLOCK / 64;

// The serial chain over p[j..cnt) (acc = the value before p[j]), numpy's
// order: two read groups alternate so the next group's LDS reads are in
// flight while the current group's adds run (as in k_scan_serial).  p is
// padded by 2 groups past cnt.  OUTG = false writes the results back into p;
// OUTG = true writes them straight to global memory at out[j..cnt) (the
// value type is the stored type: f4 / f8 little-endian), which takes the
// chain lane's LDS writes off its critical path -- measured 13.1 -> 11.0
// cycles per element for the chain alone (tools/probe_chain.py kinds 1, 14).
template <int D, bool OUTG = false>
MC_DEV typename SerAcc<D>::T fsw_chain(typename SerAcc<D>::T *p, int j, int cnt, typename SerAcc<D>::T acc,
                                       typename SerAcc<D>::T *out = nullptr) {
  using T = typename SerAcc<D>::T;
  T *o = OUTG ? out : p;
  for (; j < cnt && (j & (FSW_G - 1)); ++j) {
    acc = ser_add<D>(acc, p[j]);
    o[j] = acc;
  }
  if (j + 2 * FSW_G <= cnt) {
    T ga[FSW_G], gb[FSW_G];
    ser_ld<T, FSW_G>(p + j, ga);
    for (; j + 2 * FSW_G <= cnt; j += 2 * FSW_G) {
      ser_ld<T, FSW_G>(p + j + FSW_G, gb);
      __builtin_amdgcn_sched_barrier(0);
      acc = ser_group<D, FSW_G>(acc, ga);
      ser_st<T, FSW_G>(o + j, ga);
      ser_ld<T, FSW_G>(p + j + 2 * FSW_G, ga);
      __builtin_amdgcn_sched_barrier(0);
      acc = ser_group<D, FSW_G>(acc, gb);
      ser_st<T, FSW_G>(o + j + FSW_G, gb);
    }
  }
  for (; j < cnt; ++j) {
    acc = ser_add<D>(acc, p[j]);
    o[j] = acc;
  }
  return acc;
}

// The walker's tile layout: wave w owns the contiguous quarter
// [w*QE, (w+1)*QE) of the tile (QE = FS_Q * W * 64 elements), as FS_Q
// segments of W*64 elements with lane l's 16-B vector at W*l: every wave
// access is 1 KiB contiguous, and every predecessor except a quarter's first
// element is inside the same wave (DPP shift / readlane, no LDS).
template <int D> constexpr int fsw_qe() { return FS_Q * fs_w_of(D) * 64; }
MC_DEV int fsw_li(int q, int e, int W) {
  return (int)(threadIdx.x >> 6) * FS_Q * W * 64 + q * W * 64 + (int)(threadIdx.x & 63) * W + e;
}

// lane i <- lane i - 1 of the wave (DPP wave_shr:1; lane 0 gets `fill`)
MC_DEV uint32_t fsw_shr1(uint32_t x, uint32_t fill) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)x, 0x138, 0xF, 0xF, false);
}
template <typename S>
MC_DEV S fsw_up1(S c) {
  if constexpr (sizeof(S) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, c);
    const uint64_t r = (uint64_t)fsw_shr1((uint32_t)b, 0) | ((uint64_t)fsw_shr1((uint32_t)(b >> 32), 0) << 32);
    return __builtin_bit_cast(S, r);
  } else if constexpr (sizeof(S) == 4) {
    return __builtin_bit_cast(S, fsw_shr1(__builtin_bit_cast(uint32_t, c), 0));
  } else {
    return __builtin_bit_cast(S, (uint16_t)fsw_shr1(__builtin_bit_cast(uint16_t, c), 0));
  }
}
template <typename T>
MC_DEV T fsw_readlane(T x, int l) {  // l wave-uniform
  if constexpr (sizeof(T) == 8) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const uint64_t r = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l) << 32);
    return __builtin_bit_cast(T, r);
  } else if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint32_t, x), l));
  } else {
    return __builtin_bit_cast(T, (uint16_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint16_t, x), l));
  }
}

// branch-free select (bitwise, so the compiler keeps it a v_cndmask-free
// and/or instead of sinking an expensive operand into a branch)
template <typename T>
MC_DEV T fsw_sel(bool cond, T a, T b) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t m = 0 - (uint64_t)cond;
    return __builtin_bit_cast(T, (__builtin_bit_cast(uint64_t, a) & m) | (__builtin_bit_cast(uint64_t, b) & ~m));
  } else if constexpr (sizeof(T) == 4) {
    const uint32_t m = 0 - (uint32_t)cond;
    return __builtin_bit_cast(T, (__builtin_bit_cast(uint32_t, a) & m) | (__builtin_bit_cast(uint32_t, b) & ~m));
  } else {
    const uint16_t m = (uint16_t)(0 - (uint32_t)cond);
    return __builtin_bit_cast(T, (uint16_t)((__builtin_bit_cast(uint16_t, a) & m) |
                                            (__builtin_bit_cast(uint16_t, b) & (uint16_t)~m)));
  }
}

template <int A_, int D, int SW = 0>
MC_DEV void fsw_load(const uint8_t *src, size_t n, size_t t0, int a,
                     typename FsT<A_, D>::V (&v)[FS_Q][FsT<A_, D>::W]) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
  if constexpr (A_ == D) {  // every load first, then the swaps / conversions (see fs_load)
    typename Tr::svec xs[FS_Q];
    if (t0 + fs_tile<D>() <= n) {  // a whole tile: the loads unbranched, all in flight (see fs_load)
#pragma unroll
      for (int q = 0; q < FS_Q; ++q)
        xs[q] = __builtin_nontemporal_load(reinterpret_cast<const typename Tr::svec *>(
            src + (t0 + (size_t)fsw_li(q, 0, W)) * sizeof(typename Tr::S)));
    } else {
#pragma unroll
      for (int q = 0; q < FS_Q; ++q) {
        const size_t e0 = t0 + (size_t)fsw_li(q, 0, W);
        if (e0 + W <= n) {
          xs[q] = __builtin_nontemporal_load(
              reinterpret_cast<const typename Tr::svec *>(src + e0 * sizeof(typename Tr::S)));
        } else {
#pragma unroll
          for (int e = 0; e < W; ++e)
            xs[q][e] = e0 + e < n ? reinterpret_cast<const typename Tr::S *>(src)[e0 + e] : (typename Tr::S)0;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
      typename Tr::svec x = xs[q];
      if constexpr ((SW & 1) != 0) x = fs_bswap(x);
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = (typename Tr::V)x[e];
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    const size_t e0 = t0 + (size_t)fsw_li(q, 0, W);
    {
      const int as = mc_itemsize(a);
      uint64_t b[W];
#pragma unroll
      for (int e = 0; e < W; ++e) b[e] = e0 + e < n ? mc_load_elem_u(src, e0 + e, as) : 0;
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = e0 + e < n ? Tr::from_bits(b[e], a) : (typename Tr::V)0;
    }
  }
}

template <int A_, int D, int SW = 0>
MC_DEV void fsw_store(uint8_t *dst, size_t n, size_t t0, const typename FsT<A_, D>::S (&c)[FS_Q][FsT<A_, D>::W]) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    const size_t e0 = t0 + (size_t)fsw_li(q, 0, W);
    if (e0 + W <= n) {
      typename Tr::svec x;
#pragma unroll
      for (int e = 0; e < W; ++e) x[e] = c[q][e];
      if constexpr ((SW & 2) != 0) x = fs_bswap(x);
      __builtin_nontemporal_store(x, reinterpret_cast<typename Tr::svec *>(dst + e0 * sizeof(typename Tr::S)));
    } else {
      for (int e = 0; e < W && e0 + e < n; ++e)
        reinterpret_cast<typename Tr::S *>(dst)[e0 + e] = (SW & 2) ? fs_bswap_scalar(c[q][e]) : c[q][e];
    }
  }
}

// p[q][e] = the tile-relative inclusive double prefix of this thread's
// elements in the walker layout (any fixed association: candidates only
// propose, the per-element check decides)
template <typename V, int W, typename P>
MC_DEV void fsw_scan(const V (&v)[FS_Q][W], P (&p)[FS_Q][W], P *ldsq) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  P base = 0;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    p[q][0] = (P)v[q][0];
#pragma unroll
    for (int e = 1; e < W; ++e) p[q][e] = p[q][e - 1] + (P)v[q][e];
    const P incl = mc_wave_scan_p(p[q][W - 1]);
    const P ex = mc_wave_shr1_p(incl);
    const P pre = base + (lane ? ex : (P)0);
#pragma unroll
    for (int e = 0; e < W; ++e) p[q][e] = pre + p[q][e];
    base = base + fsw_readlane(incl, 63);
  }
  if (lane == 0) ldsq[wave] = base;  // the quarter's total
  __syncthreads();
  P off = 0;
#pragma unroll
  for (int w = 0; w < FSW_NW; ++w)
    if (w < wave) off = off + ldsq[w];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q)
#pragma unroll
    for (int e = 0; e < W; ++e) p[q][e] = off + p[q][e];
}

// The first tile >= from whose apply-time verification failed (ntiles if none).
MC_DEV size_t fsw_next_failed(const uint64_t *__restrict__ tfail, size_t from, size_t ntiles, uint64_t *ldsx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (size_t b = from; b < ntiles; b += MC_BLOCK) {
    const size_t i = b + threadIdx.x;
    const bool hit = i < ntiles && __builtin_nontemporal_load(tfail + i) != ~(uint64_t)0;
    const unsigned long long bal = __ballot(hit);
    if (lane == 0) ldsx[wave] = bal ? b + (size_t)wave * 64 + (size_t)(__ffsll(bal) - 1) : ~(uint64_t)0;
    __syncthreads();
    uint64_t m = ldsx[0];
#pragma unroll
    for (int w = 1; w < FSW_NW; ++w) m = ldsx[w] < m ? ldsx[w] : m;
    __syncthreads();
    if (m != ~(uint64_t)0) return (size_t)m;
  }
  return ntiles;
}

// Serial streaming for noise-like stretches (tiles [tb, te)): lane 0 of
// wave 0 runs numpy's chain over one tile's values in an LDS buffer while
// waves 1-3 store the previous tile's results and load the next tile into the
// other buffer (k_scan_serial's double-buffered scheme inside the walker).
// Returns the chain's value after the last element of tile te - 1.
template <int A_, int D, int SW = 0>
MC_DEV typename FsT<A_, D>::S fsw_stream(const uint8_t *src, uint8_t *dst, size_t n, int a, size_t tb, size_t te,
                                         typename FsT<A_, D>::S yin, bool has_in,
                                         typename FsT<A_, D>::V (*xs)[fs_tile_of(D) + 2 * FSW_G],
                                         typename FsT<A_, D>::S *ldsy, size_t *nan_at) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  using V = typename Tr::V;
  constexpr int W = Tr::W;
  constexpr int TE = (int)fs_tile<D>();
  constexpr int NV = TE / W;  // vectors per tile
  const int wave = threadIdx.x >> 6;
  // same-type little-endian f4 with src and dst equally 16-B aligned: wave 0
  // runs the whole stretch as one chain straight from src to dst
  // (ser_chain_vbc: no LDS staging, no per-tile barrier); the other waves
  // wait.  256 MiB of f4 noise: 294 ms against 325-360 for the LDS-fed chain
  // below; f8 stays LDS-fed (228 against 259 ms, same box,
  // profiles/r05/walk_f8_*.json)
  constexpr bool DIRECT = A_ == D && SW == 0 && D != MC_F2;
  if constexpr (DIRECT) {
    if (sizeof(S) == 4 && ((uintptr_t)src & 15) == ((uintptr_t)dst & 15)) {
      if (wave == 0) {
        const S *in = reinterpret_cast<const S *>(src);
        S *out = reinterpret_cast<S *>(dst);
        size_t e0 = tb * (size_t)TE;
        const size_t e1 = te * (size_t)TE < n ? te * (size_t)TE : n;
        V acc = Tr::val(yin);
        if (e0 == 0 && !has_in) {  // the chunk's first element: out[0] = enc[0]
          acc = in[0];
          out[0] = acc;
          e0 = 1;
        }
        acc = ser_chain_vbc<S, sizeof(S) == 8 ? 16 : 32, 6>(in + e0, out + e0, e1 - e0, acc);
        if (threadIdx.x == 0) {
          if (*nan_at == SER_NO_NAN && __builtin_isnan(acc)) *nan_at = tb * (size_t)TE;  // ser_nan_fix
          *ldsy = Tr::store(acc);
        }
      }
      __syncthreads();
      const S y = *ldsy;
      __syncthreads();  // ldsy is free again
      return y;
    }
  }
  // the I/O waves issue FSW_IOV vector loads before the first use (one at a
  // time, each waited for, the next tile's 16 KiB took longer than the
  // chain's tile and the chain lane idled at the barrier: noise-like data
  // ran 4-9 % slower than k_scan_serial)
  constexpr int FSW_IOV = 8;
  auto io_load = [&](size_t t, V *buf, int from, int step) {
    const size_t t0 = t * (size_t)TE;
    if constexpr (A_ == D) {
      for (int k0 = from; k0 < NV; k0 += FSW_IOV * step) {
        typename Tr::svec xv[FSW_IOV];
#pragma unroll
        for (int u = 0; u < FSW_IOV; ++u) {
          const int k = k0 + u * step;
          const size_t e0 = t0 + (size_t)k * W;
          if (k < NV && e0 + W <= n) {
            xv[u] = __builtin_nontemporal_load(reinterpret_cast<const typename Tr::svec *>(src + e0 * sizeof(S)));
            if constexpr ((SW & 1) != 0) xv[u] = fs_bswap(xv[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < FSW_IOV; ++u) {
          const int k = k0 + u * step;
          const size_t e0 = t0 + (size_t)k * W;
          if (k >= NV) continue;
          if (e0 + W <= n) {
#pragma unroll
            for (int e = 0; e < W; ++e) buf[k * W + e] = (V)xv[u][e];
          } else {
#pragma unroll
            for (int e = 0; e < W; ++e)
              buf[k * W + e] = e0 + e < n ? Tr::from_bits(mc_load_elem_u(src, e0 + e, sizeof(S)), a) : (V)0;
          }
        }
      }
      return;
    }
    for (int k = from; k < NV; k += step) {
      const size_t e0 = t0 + (size_t)k * W;
      const int as = mc_itemsize(a);
#pragma unroll
      for (int e = 0; e < W; ++e)
        buf[k * W + e] = e0 + e < n ? Tr::from_bits(mc_load_elem_u(src, e0 + e, as), a) : (V)0;
    }
  };
  auto io_store = [&](size_t t, const V *buf, int from, int step) {
    const size_t t0 = t * (size_t)TE;
    for (int k = from; k < NV; k += step) {
      const size_t e0 = t0 + (size_t)k * W;
      if (e0 >= n) break;
      if (e0 + W <= n) {
        typename Tr::svec x;
#pragma unroll
        for (int e = 0; e < W; ++e) x[e] = Tr::store(buf[k * W + e]);
        if constexpr ((SW & 2) != 0) x = fs_bswap(x);
        __builtin_nontemporal_store(x, reinterpret_cast<typename Tr::svec *>(dst + e0 * sizeof(S)));
      } else {
        for (int e = 0; e < W && e0 + e < n; ++e) {
          const S c = Tr::store(buf[k * W + e]);
          reinterpret_cast<S *>(dst)[e0 + e] = (SW & 2) ? fs_bswap_scalar(c) : c;
        }
      }
    }
  };
  io_load(tb, xs[tb & 1], threadIdx.x, MC_BLOCK);
  __syncthreads();
  V acc = Tr::val(yin);
  for (size_t t = tb; t < te; ++t) {
    if (wave == 0) {
      if (threadIdx.x == 0) {
        const size_t t0 = t * (size_t)TE;
        const int cnt = (int)(n - t0 < (size_t)TE ? n - t0 : (size_t)TE);
        V *p = xs[t & 1];
        int j = 0;
        V *out = reinterpret_cast<V *>(dst + t0 * sizeof(S));
        if (t0 == 0 && !has_in) {  // the chunk's first element: out[0] = enc[0]
          acc = p[0];
          if constexpr (DIRECT) out[0] = acc;
          j = 1;
        }
        if constexpr (DIRECT) acc = fsw_chain<D, true>(p, j, cnt, acc, out);
        else acc = fsw_chain<D>(p, j, cnt, acc);
        if (D != MC_F2 && *nan_at == SER_NO_NAN && __builtin_isnan(acc)) *nan_at = t0;  // ser_nan_fix
        if (t + 1 == te) *ldsy = Tr::store(acc);
      }
    } else {
      const int io = threadIdx.x - 64;
      if (!DIRECT && t > tb) io_store(t - 1, xs[(t - 1) & 1], io, MC_BLOCK - 64);
      if (t + 1 < te) io_load(t + 1, xs[(t + 1) & 1], io, MC_BLOCK - 64);
    }
    __syncthreads();
  }
  if (!DIRECT) io_store(te - 1, xs[(te - 1) & 1], threadIdx.x, MC_BLOCK);
  const S y = *ldsy;
  __syncthreads();  // the buffers and ldsy are free again
  return y;
}

template <int A_, int D, int SW = 0>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_walk(const uint8_t *__restrict__ src, size_t src_stride,
                                                        uint8_t *__restrict__ dst, size_t dst_stride, size_t n,
                                                        int a, uint64_t *__restrict__ rowfail,
                                                        const double *__restrict__ sums,
                                                        const double *__restrict__ pre,
                                                        const uint64_t *__restrict__ tfail,
                                                        const uint64_t *__restrict__ fail) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  using V = typename Tr::V;
  using P = typename Tr::P;
  constexpr int W = Tr::W;
  constexpr int TE = (int)fs_tile<D>();
  constexpr int QE = fsw_qe<D>();
  constexpr int NOFAIL = 0x7fffffff;
  // per pass, each wave publishes its last candidate, its first element
  // (value, candidate, prefix) and its first failure inside the quarter
  __shared__ P ldsq[FSW_NW];
  __shared__ S lds_last[2][FSW_NW], lds_bc[2][FSW_NW], lds_fv[2][FSW_NW];
  __shared__ V lds_bv[2][FSW_NW];
  __shared__ P lds_bp[2][FSW_NW], lds_fp[2][FSW_NW];
  __shared__ int lds_fi[2][FSW_NW];
  __shared__ uint64_t ldsx[FSW_NW];
  __shared__ S ldsy;
  __shared__ size_t nan_at;              // first tile whose chain ended NaN (ser_nan_fix)
  __shared__ unsigned long long nan_k0;
  __shared__ __attribute__((aligned(16))) V xs2[2][TE + 2 * FSW_G];
  V *xs = xs2[0];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool single = sums != nullptr;
  src += (size_t)blockIdx.x * src_stride;
  dst += (size_t)blockIdx.x * dst_stride;
  const size_t ntiles = (n + TE - 1) / TE;
  size_t t = 0;
  bool has_in = false;
  S yin = (S)0;
  if (threadIdx.x == 0) nan_at = SER_NO_NAN;  // published by the loop's first barrier
  if (single) {
    const uint64_t f = *fail;  // the first index that failed at apply time
    if (f >= n) return;        // everything verified: dst is final
    t = (size_t)(f / TE);
    has_in = t > 0;
    if (has_in) yin = Tr::bound(pre[t - 1], sums[t - 1]);  // tile t-1 verified: its last candidate
  } else {
    // a row that k_fspec_rows left at its first failing tile (rowfail = its
    // start; n when the row verified): resume there from the last stored value
    const uint64_t f = rowfail[blockIdx.x];
    if (f >= n) return;
    t = (size_t)(f / TE);
    has_in = t > 0;
    if (has_in) {
      yin = reinterpret_cast<const S *>(dst)[t * (size_t)TE - 1];
      if constexpr ((SW & 2) != 0) yin = fs_bswap_scalar(yin);
    }
  }
  int serial_run = 0, par = 0;
  size_t next_probe = 0, gap = FSW_PROBE;  // serial tiles stream until next_probe
  V nv[FS_Q][W];
  fsw_load<A_, D, SW>(src, n, t * TE, a, nv);
  while (t < ntiles) {
    if (serial_run > 0 && t < next_probe) {
      // noise-like stretch: serial streaming up to the next probe tile
      const size_t te = next_probe < ntiles ? next_probe : ntiles;
      yin = fsw_stream<A_, D, SW>(src, dst, n, a, t, te, yin, has_in, xs2, &ldsy, &nan_at);
      has_in = true;
      serial_run += (int)(te - t);
      t = te;
      if (t >= ntiles) break;
      fsw_load<A_, D, SW>(src, n, t * (size_t)TE, a, nv);
      if (single && Tr::bits(yin) == Tr::bits(Tr::bound(pre[t - 1], sums[t - 1]))) {
        const size_t nt = fsw_next_failed(tfail, t, ntiles, ldsx);
        if (nt >= ntiles) break;
        if (nt != t) {
          t = nt;
          yin = Tr::bound(pre[nt - 1], sums[nt - 1]);
          fsw_load<A_, D, SW>(src, n, nt * (size_t)TE, a, nv);
        }
        serial_run = 0;
        gap = FSW_PROBE;
      }
      continue;
    }
    const size_t t0 = t * (size_t)TE;
    V v[FS_Q][W];
#pragma unroll
    for (int q = 0; q < FS_Q; ++q)
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = nv[q][e];
    if (t + 1 < ntiles) fsw_load<A_, D, SW>(src, n, t0 + TE, a, nv);  // the usual successor, in flight
    const int cnt = (int)(n - t0 < (size_t)TE ? n - t0 : (size_t)TE);
    const bool first_tile = t0 == 0;
    S c[FS_Q][W];
    int fpos = -1;  // elements at local index <= fpos are final
    S fixed = yin;  // the true value at fpos
    bool go_serial = false;
    const int cap = serial_run > 0 ? FSW_PROBE_CAP : FSW_CAP;
    if (!go_serial) {
      P p[FS_Q][W];
      fsw_scan<V, W, P>(v, p, ldsq);
      // candidates c_i = D(kb + p_i) with kb = y_base - p_base (one add per
      // element; any association proposes, the check decides)
      P kb = has_in ? (P)Tr::val(yin) : (P)0;
      int steps = 0;
      for (;; par ^= 1) {
        // candidates (branch-free: every element computes, selects keep the
        // final ones)
#pragma unroll
        for (int q = 0; q < FS_Q; ++q) {
#pragma unroll
          for (int e = 0; e < W; ++e) {
            const int li = fsw_li(q, e, W);
            const S cn = Tr::round(kb + p[q][e]);
            c[q][e] = fsw_sel(li > fpos, cn, fsw_sel(li == fpos, fixed, c[q][e]));
          }
        }
        // every predecessor inside the wave; the quarter's first element is
        // checked after the barrier (its predecessor is the previous wave's).
        // Descending order, so the smallest failing index is selected last.
        uint32_t bm = 0;  // bit q*W+e: element (q, e) fails
        S pvs[FS_Q];
        {
          S prevseg = (S)0;
#pragma unroll
          for (int q = 0; q < FS_Q; ++q) {
            const S up = fsw_up1(c[q][W - 1]);
            pvs[q] = lane ? up : prevseg;
            prevseg = fsw_readlane(c[q][W - 1], 63);
          }
        }
#pragma unroll
        for (int q = 0; q < FS_Q; ++q) {
#pragma unroll
          for (int e = 0; e < W; ++e) {
            const int li = fsw_li(q, e, W);
            const S pe = e ? c[q][e - 1] : pvs[q];
            const S r = Tr::store(Tr::step(Tr::val(pe), v[q][e]));
            // non-short-circuit (&): no control flow per element
            const bool ok = (int)(Tr::bits(c[q][e]) == Tr::bits(r)) & (int)Tr::finite(c[q][e]);
            const bool bad = (!ok) & (li > fpos) & (li < cnt) & !(q == 0 && e == 0 && lane == 0);
            bm |= (uint32_t)bad << (q * W + e);
          }
        }
        // the wave's smallest failing index: lanes own interleaved vectors,
        // so it is the lowest failing lane of the lowest segment q; its
        // corrected value is recomputed once, by a switch on the (uniform)
        // element position of that lane
        int wf = NOFAIL;
        S wv = (S)0;
        P wp = 0;
        if (__ballot(bm != 0)) {
          int fl = 0, fk = 0;
#pragma unroll
          for (int q = FS_Q - 1; q >= 0; --q) {
            const unsigned long long bal = __ballot((bm >> (q * W)) & ((1u << W) - 1));
            if (bal) {
              fl = __ffsll(bal) - 1;
              fk = __builtin_ctz(((uint32_t)__builtin_amdgcn_readlane((int)bm, fl) >> (q * W))) + q * W;
            }
          }
          S r = (S)0;
          P pk = 0;
#pragma unroll
          for (int k = 0; k < FS_Q * W; ++k) {
            if (k == fk) {  // uniform
              const int q = k / W, e = k % W;
              const S pe = e ? c[q][e - 1] : pvs[q];
              r = Tr::store(Tr::step(Tr::val(pe), v[q][e]));
              pk = p[q][e];
            }
          }
          wf = wave * QE + (fk / W) * W * 64 + fl * W + fk % W;
          wv = fsw_readlane(r, fl);
          wp = fsw_readlane(pk, fl);
        }
        if (lane == 63) lds_last[par][wave] = c[FS_Q - 1][W - 1];
        if (lane == 0) {
          lds_bc[par][wave] = c[0][0];
          lds_bv[par][wave] = v[0][0];
          lds_bp[par][wave] = p[0][0];
          lds_fi[par][wave] = wf;
          lds_fv[par][wave] = wv;
          lds_fp[par][wave] = wp;
        }
        __syncthreads();
        // uniform: the quarters' first elements and the waves' first
        // failures, from the last quarter down so the smallest index is
        // selected last (all LDS reads independent)
        int f = NOFAIL;
        S fv = (S)0;
        P fp = 0;
#pragma unroll
        for (int w = FSW_NW - 1; w >= 0; --w) {
          const int wfi = lds_fi[par][w];
          const S wfv = lds_fv[par][w], bc = lds_bc[par][w];
          const P wfp = lds_fp[par][w], bp = lds_bp[par][w];
          const V bv = lds_bv[par][w];
          const S pe = w ? lds_last[par][w - 1] : yin;  // w = 0: only checked while fpos < 0
          f = fsw_sel(wfi != NOFAIL, wfi, f);
          fv = fsw_sel(wfi != NOFAIL, wfv, fv);
          fp = fsw_sel(wfi != NOFAIL, wfp, fp);
          const int lb = w * QE;
          const S r = Tr::store((w == 0 && first_tile) ? bv : Tr::step(Tr::val(pe), bv));  // out[0] = enc[0]
          const bool bad = (lb > fpos) & (lb < cnt) & !((int)(Tr::bits(bc) == Tr::bits(r)) & (int)Tr::finite(bc));
          f = fsw_sel(bad, lb, f);
          fv = fsw_sel(bad, r, fv);
          fp = fsw_sel(bad, bp, fp);
        }
        if (f == NOFAIL) break;  // the tile verified from the true values before it
        // re-base at f: numpy's value there (its predecessor is verified)
        fpos = f;
        fixed = fv;
        kb = (P)Tr::val(fv) - fp;
        if (++steps >= cap) {
          go_serial = true;
          break;
        }
      }
    }
    if (go_serial) {
      // serial fallback: the tile's values in element order in LDS, one lane
      // runs numpy's chain from the last true value, every lane reads back
#pragma unroll
      for (int q = 0; q < FS_Q; ++q)
#pragma unroll
        for (int e = 0; e < W; ++e) xs[fsw_li(q, e, W)] = v[q][e];
      __syncthreads();
      if (threadIdx.x == 0) {
        int j = fpos + 1;
        V acc;
        if (fpos >= 0) acc = Tr::val(fixed);
        else if (has_in) acc = Tr::val(yin);
        else {  // the chunk's first element: out[0] = enc[0]
          acc = xs[0];
          j = 1;
        }
        const V last = fsw_chain<D>(xs, j, cnt, acc);
        ldsy = Tr::store(last);
        if (D != MC_F2 && nan_at == SER_NO_NAN && __builtin_isnan(last)) nan_at = t0;  // ser_nan_fix
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < FS_Q; ++q)
#pragma unroll
        for (int e = 0; e < W; ++e) {
          const int li = fsw_li(q, e, W);
          if (li > fpos) c[q][e] = Tr::store(xs[li]);
          else if (li == fpos) c[q][e] = fixed;
        }
      if (serial_run > 0) gap = gap * 2 < (size_t)FSW_PROBE_MAX ? gap * 2 : (size_t)FSW_PROBE_MAX;  // probe failed
      ++serial_run;
      next_probe = t + gap;
      yin = ldsy;
    } else {
      serial_run = 0;
      gap = FSW_PROBE;
      yin = lds_last[par][FSW_NW - 1];  // the tile's last element (full tiles)
      par ^= 1;
    }
    has_in = true;
    fsw_store<A_, D, SW>(dst, n, t0, c);
    if (t + 1 >= ntiles) break;
    if (single && Tr::bits(yin) == Tr::bits(Tr::bound(pre[t], sums[t]))) {
      // in sync with the apply pass: tiles that verified there are final
      const size_t nt = fsw_next_failed(tfail, t + 1, ntiles, ldsx);
      if (nt >= ntiles) break;
      if (nt != t + 1) {
        t = nt;
        yin = Tr::bound(pre[nt - 1], sums[nt - 1]);
        fsw_load<A_, D, SW>(src, n, nt * (size_t)TE, a, nv);
        continue;
      }
    }
    ++t;
  }
  if constexpr (D != MC_F2) {  // numpy's NaN tail (f2 chains are exact in-chain)
    __syncthreads();
    if (nan_at != SER_NO_NAN)
      ser_nan_fix<D>(src, a, dst, D | ((SW & 2) != 0 ? MC_BIG_ENDIAN : 0), n, nan_at, &nan_k0);
  }
}

// Tile prefixes by many workgroups (one per 256 tiles): workgroup g sums
// all totals before its range itself (coalesced, 8 loads in flight per
// thread) and scans its own 256.  A one-workgroup scan (LDS-staged, 4096
// totals per round) was bound by a single CU's bandwidth: 14.7 us for
// 16 Ki tiles against 7.9 us here (6.6 us since round 4, 32 loads in flight
// per thread instead of 8); reading the earlier totals redundantly
// spreads that over ntiles/256 CUs.  Any association is
// fine: the apply pass only relies on the stored pre[] and sums[].
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_pre(const double *__restrict__ sums,
                                                       double *__restrict__ pre, size_t ntiles,
                                                       uint64_t *__restrict__ tfail,
                                                       uint64_t *__restrict__ fail, size_t n) {
  __shared__ double lds[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t b = (size_t)blockIdx.x * MC_BLOCK;
  // 32 loads in flight per thread per round trip (8 took ~8 round trips
  // for the last workgroup of 16 Ki tiles: 8.2 us for the whole kernel)
  constexpr int PU = 32;
  double a[PU];
#pragma unroll
  for (int k = 0; k < PU; ++k) a[k] = 0.0;
  for (size_t i = threadIdx.x; i < b; i += PU * MC_BLOCK) {
    double v[PU];  // branch-free: every load issued before the adds
#pragma unroll
    for (int k = 0; k < PU; ++k) {
      const size_t j = i + (size_t)k * MC_BLOCK;
      v[k] = sums[j < b ? j : b - 1];
    }
#pragma unroll
    for (int k = 0; k < PU; ++k) a[k] += i + (size_t)k * MC_BLOCK < b ? v[k] : 0.0;
  }
#pragma unroll
  for (int h = PU / 2; h > 0; h >>= 1)
#pragma unroll
    for (int k = 0; k < h; ++k) a[k] += a[k + h];
  double acc = a[0];
  const double x = b + threadIdx.x < ntiles ? sums[b + threadIdx.x] : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  double incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double o = __shfl_up(incl, off, 64);
    if (lane >= off) incl = o + incl;
  }
  const double ex = __shfl_up(incl, 1, 64);
  if (lane == 0) lds[0][wave] = acc;
  if (lane == 63) lds[1][wave] = incl;
  __syncthreads();
  double base = 0.0, w = 0.0;
#pragma unroll
  for (int j = 0; j < MC_BLOCK / 64; ++j) {
    base += lds[0][j];
    if (j < wave) w += lds[1][j];
  }
  if (b + threadIdx.x < ntiles) {
    pre[b + threadIdx.x] = base + (w + (lane ? ex : 0.0));
    tfail[b + threadIdx.x] = ~(uint64_t)0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *fail = n;
}

// Workspace (fspec_ws_bytes): sums, pre, tfail (ntiles words each), then
// fail (the last word).  `ticket` is unused: every arrival-ticket schedule
// measured slower (above).
template <int A_, int D, int SW = 0>
static void launch_fspec(const uint8_t *s, uint8_t *d, size_t n, int a, void *ws, uint32_t *ticket, hipStream_t st) {
  (void)ticket;
  const size_t ntiles = fspec_ntiles(n, D);
  double *sums = static_cast<double *>(ws), *pre = sums + ntiles;
  uint64_t *tfail = reinterpret_cast<uint64_t *>(pre + ntiles), *fail = tfail + ntiles;
  k_fspec_reduce<A_, D, SW><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, n, a, sums);
  k_fspec_pre<<<(unsigned)((ntiles + MC_BLOCK - 1) / MC_BLOCK), MC_BLOCK, 0, st>>>(sums, pre, ntiles, tfail, fail, n);
  k_fspec_apply<A_, D, SW><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, a, sums, pre, tfail, fail);
  // one walker from the first failing tile (returns at once if none failed)
  k_fspec_walk<A_, D, SW><<<1, MC_BLOCK, 0, st>>>(s, 0, d, 0, n, a, nullptr, sums, pre, tfail, fail);
}

// the speculative rows pass, then one walker per row that failed (rows that
// verified return at once)
template <int A_, int D, int SW = 0>
static void launch_fspec_rows(const uint8_t *sc, size_t src_stride, uint8_t *dc, size_t dst_stride, size_t n, int a,
                              uint64_t *fail, unsigned g, hipStream_t st) {
  k_fspec_rows<A_, D, SW><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n, a, fail);
  k_fspec_walk<A_, D, SW><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n, a, fail, nullptr, nullptr,
                                                nullptr, nullptr);
}

}  // namespace
