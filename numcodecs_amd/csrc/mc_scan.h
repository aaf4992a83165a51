// mc_scan.h -- block/wave scan building blocks shared by the Delta decode
// scan (mc_scan.hip) and the fused FSO->Delta->Shuffle decode (mc_c4.hip).
// (The single-pass decoupled look-back schedules measured against these
// live in tools/lab/, outside the product library.)
#pragma once

#include "mc_num.h"

constexpr int MC_SCAN_STEPS = 4;
constexpr int MC_SCAN_TILE = 4 * MC_SCAN_STEPS * MC_BLOCK;  // 4096 elements

template <bool OR_OP>
MC_DEV uint64_t mc_scan_combine(uint64_t a, uint64_t b) {
  if constexpr (OR_OP) return a | b;
  else return a + b;
}

template <bool OR_OP>
MC_DEV uint64_t mc_wave_incl_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t o = __shfl_up(v, off, 64);
    if (lane >= off) v = mc_scan_combine<OR_OP>(v, o);
  }
  return v;
}

// Exclusive scan across the blockDim.x (<= 1024) threads of a block: returns
// this thread's exclusive prefix; *total = block total.  `lds` holds
// blockDim.x/64 words.  Contains two __syncthreads().
template <bool OR_OP>
MC_DEV uint64_t mc_block_excl_scan(uint64_t v, uint64_t *lds, uint64_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = (blockDim.x + 63) >> 6;
  const uint64_t incl = mc_wave_incl_scan<OR_OP>(v);
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  uint64_t wpre = 0, tot = 0;
  for (int w = 0; w < nwaves; ++w) {
    const uint64_t x = lds[w];
    if (w < wave) wpre = mc_scan_combine<OR_OP>(wpre, x);
    tot = mc_scan_combine<OR_OP>(tot, x);
  }
  __syncthreads();
  *total = tot;
  const uint64_t excl_in_wave = __shfl_up(incl, 1, 64);
  return mc_scan_combine<OR_OP>(wpre, lane ? excl_in_wave : 0);
}

// 32-bit exclusive block sum scan (mod 2^32): half the shuffle traffic of the
// 64-bit mc_block_excl_scan for callers whose totals are 32-bit (the int16 /
// int32 C4 scan).  Same contract: two __syncthreads(), `lds` holds
// blockDim.x/64 words.
MC_DEV uint32_t mc_block_excl_scan32(uint32_t v, uint32_t *lds, uint32_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = (blockDim.x + 63) >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  uint32_t wpre = 0, tot = 0;
  for (int w = 0; w < nwaves; ++w) {
    const uint32_t x = lds[w];
    if (w < wave) wpre += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  const uint32_t excl_in_wave = __shfl_up(incl, 1, 64);
  return wpre + (lane ? excl_in_wave : 0u);
}

// Exclusive scan of `ntiles` tile totals in place, one workgroup of 1024
// (tools/scan_bench.hip measures it alone).  Per round of 8192 totals each
// wave moves its 512 through an LDS slice with coalesced global accesses
// (lane l loads l + 64k) and scans them as 8 consecutive totals per lane
// (serial adds), so one block scan -- one wave scan per wave -- is all the
// cross-lane work.  Two layouts measured slower: 16 consecutive totals per
// lane straight from global (each load instruction touches 64 cache lines on
// one CU: 18.7 us for 16K totals), 64-lane columns scanned across the wave
// (16 wave scans of 64-bit shuffles per round: 15.5 us) and 16K-total rounds
// (a 128 KiB LDS workgroup adds ~4 us of fixed cost).  This one: 9.2 us for
// 16K totals, 4.8 us for one round, the next round's loads issued early.
template <bool OR_OP>
__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t *__restrict__ sums, size_t ntiles) {
  constexpr int PER = 8, WSPAN = 64 * PER, ROUND = 1024 * PER;  // 64 KiB LDS
  __shared__ uint64_t red[1024 / 64];
  __shared__ __attribute__((aligned(16))) uint64_t buf[ROUND];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t *wbuf = buf + wave * WSPAN;
  uint64_t carry = 0;
  const size_t last = ntiles - 1;
  uint64_t x[PER];  // this round's totals; the next round's are loaded early
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const size_t i = (size_t)wave * WSPAN + lane + 64 * k;
    x[k] = sums[i < last ? i : last];
  }
  for (size_t r0 = 0; r0 < ntiles; r0 += ROUND) {
    const size_t wb = r0 + (size_t)wave * WSPAN + lane;
    uint64_t xn[PER];
    if (r0 + ROUND < ntiles) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const size_t i = wb + ROUND + 64 * k;
        xn[k] = sums[i < last ? i : last];
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) wbuf[lane + 64 * k] = wb + 64 * k < ntiles ? x[k] : 0;
    // the wave reads back what it wrote: no barrier needed, only LDS ordering
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    uint64_t v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = wbuf[PER * lane + k];
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint64_t t = v[k];
      v[k] = run;
      run = mc_scan_combine<OR_OP>(run, t);
    }
    uint64_t tot;
    const uint64_t excl = mc_scan_combine<OR_OP>(carry, mc_block_excl_scan<OR_OP>(run, red, &tot));
#pragma unroll
    for (int k = 0; k < PER; ++k) wbuf[PER * lane + k] = mc_scan_combine<OR_OP>(excl, v[k]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (wb + 64 * k < ntiles) sums[wb + 64 * k] = wbuf[lane + 64 * k];
    carry = mc_scan_combine<OR_OP>(carry, tot);
    if (r0 + ROUND < ntiles) {
#pragma unroll
      for (int k = 0; k < PER; ++k) x[k] = xn[k];
    }
  }
}

template <bool OR_OP>
static inline void mc_launch_scan_sums(uint64_t *sums, size_t ntiles, hipStream_t st) {
  k_scan_sums<OR_OP><<<1, 1024, 0, st>>>(sums, ntiles);
}

// Exclusive scan of n totals into a separate array by one workgroup per 256
// totals: workgroup g combines every total before its range itself
// (coalesced, 8 loads in flight per thread) and scans its own 256.  The
// one-workgroup k_scan_sums is bound by a single CU (4.8 us for one round of
// 8192, ~8 us in the C4 decode); reading the earlier totals redundantly
// spreads the work over n/256 CUs.  Not in place (in != out).
template <bool OR_OP>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_sums_mw(const uint64_t *__restrict__ in,
                                                          uint64_t *__restrict__ out, size_t n) {
  __shared__ uint64_t red[MC_BLOCK / 64];
  __shared__ uint64_t base_lds[MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t b = (size_t)blockIdx.x * MC_BLOCK;
  uint64_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t i = threadIdx.x;
  for (; i + 7 * MC_BLOCK < b; i += 8 * MC_BLOCK) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = mc_scan_combine<OR_OP>(a[k], in[i + (size_t)k * MC_BLOCK]);
  }
  for (; i < b; i += MC_BLOCK) a[0] = mc_scan_combine<OR_OP>(a[0], in[i]);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) acc = mc_scan_combine<OR_OP>(acc, a[k]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc = mc_scan_combine<OR_OP>(acc, __shfl_xor(acc, off, 64));
  if (lane == 0) base_lds[wave] = acc;
  const uint64_t x = b + threadIdx.x < n ? in[b + threadIdx.x] : 0;
  uint64_t tot;
  const uint64_t ex = mc_block_excl_scan<OR_OP>(x, red, &tot);  // its barriers publish base_lds
  uint64_t base = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) base = mc_scan_combine<OR_OP>(base, base_lds[w]);
  if (b + threadIdx.x < n) out[b + threadIdx.x] = mc_scan_combine<OR_OP>(base, ex);
}

template <bool OR_OP>
static inline void mc_launch_scan_sums_mw(const uint64_t *in, uint64_t *out, size_t n, hipStream_t st) {
  k_scan_sums_mw<OR_OP><<<(unsigned)((n + MC_BLOCK - 1) / MC_BLOCK), MC_BLOCK, 0, st>>>(in, out, n);
}

// ---------------------------------------------------------------------------
// Float Delta decode pieces shared by the serial chain (mc_scan.hip) and the
// speculative path (mc_fspec.h, mc_fspec_f2/f4/f8.hip).
// ---------------------------------------------------------------------------
template <int D> struct SerAcc { using T = float; };
template <> struct SerAcc<MC_F8> { using T = double; };

// numpy's add of the running sum a and the next value b in D's loop type.
// f2: numpy's half loop, float32 add then npy_float_to_half (the hardware RNE
// conversion, with denormals kept, gives the same half for every non-NaN
// sum; NaN sums take numpy's payload-preserving routine and its operand
// choice: the half loop keeps the SECOND operand's NaN when both are NaN --
// measured, cumsum([NaN_a, NaN_b]) gives NaN_b for float16).  f4 / f8: the
// plain IEEE add; where the running sum turns NaN the GPU's NaN bits differ
// from numpy's (x86 keeps the first operand's NaN, and inf + -inf is the
// negative default NaN there), and the chain kernels rewrite that NaN tail
// afterwards (ser_nan_fix) instead of paying for it on the critical path.
template <int D>
MC_DEV typename SerAcc<D>::T ser_add(typename SerAcc<D>::T a, typename SerAcc<D>::T b) {
  if constexpr (D == MC_F2) {
    const float r = a + b;
    if (__builtin_isnan(r)) return mc_half_to_float(mc_float_to_half(mc_x86_nan(b, a, r)));
    return (float)(_Float16)r;
  } else {
    return a + b;
  }
}

// One group of the chain, in place (g[k] <- the running sum after g[k]).
// f2: numpy adds in float32 and rounds to half; with float32's 24 >= 2*11+2
// bits that double rounding equals one correctly rounded half add, so the
// group runs as a chain of half adds (v_add_f16, one dependent op per
// element; LLVM folds the float<->half round trips between them).  NaN is
// absorbing in the chain, so a group ending in NaN is recomputed with the
// exact routine (ser_add: numpy's payload-preserving conversion and NaN
// choice) from its first value.  f4 / f8: plain dependent adds (NaN tails:
// ser_nan_fix).
template <int D, int G>
MC_DEV typename SerAcc<D>::T ser_group(typename SerAcc<D>::T acc, typename SerAcc<D>::T (&g)[G]) {
  using T = typename SerAcc<D>::T;
  if constexpr (D == MC_F2) {
    const T a0 = acc;
    T r[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      acc = (float)((_Float16)acc + (_Float16)g[k]);
      r[k] = acc;
    }
    if (__builtin_isnan(acc)) {
      acc = a0;
#pragma unroll
      for (int k = 0; k < G; ++k) {
        acc = ser_add<D>(acc, g[k]);
        r[k] = acc;
      }
    }
#pragma unroll
    for (int k = 0; k < G; ++k) g[k] = r[k];
  } else {
#pragma unroll
    for (int k = 0; k < G; ++k) {
      acc = ser_add<D>(acc, g[k]);
      g[k] = acc;
    }
  }
  return acc;
}

// ---------------------------------------------------------------------------
// The chain fed through VGPRs by uniform-address vector loads (round 5): every
// lane of the calling wave loads the same 16 B per instruction, runs the same
// dependent adds on VGPR operands and stores the same results as 16-B
// vectors -- no lane-0 branch and no LDS staging of the inputs.  Vector loads
// return in order, so D groups of SG values stay in flight (the compiler's
// vmcnt(N) waits only for the group about to be added), which hides HBM's
// latency without a prefetching wave.  In the product's noise-like float32
// Delta decode (k_fspec_walk, 256 MiB) it runs at 294 ms against 325-360 ms
// for the LDS-fed lane-0 chain and 325 ms for a scalar-load (SGPR operand)
// chain with an L2-prefetching wave (tools/lab/lab_chain.hip,
// tools/probe_stream.py).  The scalar chain is the fastest on cache-resident
// input (lab kinds 23 / 42), but scalar loads return out of order (any wait
// is lgkmcnt(0)), so it keeps only one group in flight and its per-group L2
// latency bounds it when streaming.  For float64 the LDS-fed chain stays
// faster in the walker (228 vs 259 ms on one box): the all-lane 16-B loads
// and stores, one per two elements, cost more issue time than its lane-0
// LDS reads.  `in` and `out` must have the same address modulo 16 (the
// callers check).
// ---------------------------------------------------------------------------
template <typename T, int SG, int D>
MC_DEV T ser_chain_vbc(const T *in, T *out, size_t cnt, T acc) {
  constexpr int W = 16 / (int)sizeof(T);
  typedef T vec __attribute__((ext_vector_type(W)));
  typedef __attribute__((address_space(1))) T *gp;
  typedef __attribute__((address_space(1))) vec *gvp;
  typedef const __attribute__((address_space(1))) vec *cgvp;
  typedef const __attribute__((address_space(1))) T *cgp;
  int z;  // a zero the compiler cannot prove uniform: the loads stay vector loads
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  const cgp src = (cgp)(in + z);
  const gp dstp = (gp)mc_uniform_ptr(out);
  // a short run [j, j + m) (m <= SG), its loads issued together
  auto run = [&](size_t j, int m) {
    T v[SG];
#pragma unroll
    for (int k = 0; k < SG; ++k) v[k] = k < m ? src[j + k] : (T)0;
#pragma unroll
    for (int k = 0; k < SG; ++k)
      if (k < m) {
        acc = acc + v[k];
        dstp[j + k] = acc;
      }
  };
  size_t j = 0;
  {
    const int h = (int)(((16 - ((uintptr_t)out & 15)) & 15) / sizeof(T));
    const int m = (size_t)h < cnt ? h : (int)cnt;
    if (m > 0) run(0, m);
    j = m;
  }
  auto ld = [&](size_t at, T(&g)[SG]) {
    const cgvp q = (cgvp)(src + at);
#pragma unroll
    for (int k = 0; k < SG / W; ++k) {
      const vec x = q[k];
#pragma unroll
      for (int e = 0; e < W; ++e) g[W * k + e] = x[e];
    }
  };
  auto grp = [&](size_t at, const T(&g)[SG]) {
    T res[SG];
#pragma unroll
    for (int k = 0; k < SG; ++k) {
      acc = acc + g[k];
      res[k] = acc;
    }
    const gvp o = (gvp)(dstp + at);
#pragma unroll
    for (int k = 0; k < SG / W; ++k) {
      vec x;
#pragma unroll
      for (int e = 0; e < W; ++e) x[e] = res[W * k + e];
      o[k] = x;
    }
  };
  if (j + (size_t)D * SG <= cnt) {
    T buf[D][SG];
#pragma unroll
    for (int u = 0; u < D; ++u) ld(j + (size_t)u * SG, buf[u]);
    for (; j + 2 * (size_t)D * SG <= cnt; j += (size_t)D * SG) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        grp(j + (size_t)u * SG, buf[u]);
        ld(j + (size_t)(u + D) * SG, buf[u]);
      }
    }
    // the last loaded round, the remaining whole groups loaded behind it
    const size_t j2 = j + (size_t)D * SG;
    const int ng = (int)((cnt - j2) / SG);  // < D
#pragma unroll
    for (int u = 0; u < D; ++u) {
      grp(j + (size_t)u * SG, buf[u]);
      if (u < ng) ld(j2 + (size_t)u * SG, buf[u]);
    }
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (u < ng) grp(j2 + (size_t)u * SG, buf[u]);
    j = j2 + (size_t)ng * SG;
  }
  for (; j < cnt; j += SG) run(j, cnt - j < (size_t)SG ? (int)(cnt - j) : SG);
  return acc;
}

// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// numpy's NaN tail of a float32 / float64 cumsum.  NaN is absorbing, so
// every running sum from the first NaN one (index k0) on is NaN, and numpy's
// loop (x86: the first operand's NaN is kept, quieted) makes them all equal
// to the first: the NaN input at k0 quieted (a finite sum + NaN), the
// negative default NaN (inf + -inf), or -- k0 = 0, the first element, which
// is copied without an add -- that input quieted from k0 + 1 on.  A chain
// kernel whose running sum ended NaN in some block calls ser_nan_fix once at
// its end, with every thread of the workgroup, from the start of the first
// such block: it finds k0 in dst and rewrites [k0, n) (or [1, n)) with those
// bits, cast to the output dtype d (whose bits it writes as stored).
// ---------------------------------------------------------------------------
MC_DEV bool ser_is_nan_bits(uint64_t b, int d) {
  switch (mc_dt_base(d)) {
    case MC_F2: return (b & 0x7fffu) > 0x7c00u;
    case MC_F4: return (b & 0x7fffffffu) > 0x7f800000u;
    default: return (b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
  }
}

template <int L>
MC_DEV uint64_t ser_nan_tail_bits(uint64_t e_bits, int a, int d) {
  static_assert(L == MC_F4 || L == MC_F8, "float32 / float64 loops");
  const McNum v = mc_num_cast(mc_num_from_bits(e_bits, a), a, L);
  double q;
  if (L == MC_F4) {
    const uint32_t b = __builtin_isnan(v.f) ? (mc_f32_bits((float)v.f) | 0x00400000u) : 0xFFC00000u;
    q = (double)mc_bits_f32(b);
  } else {
    q = mc_bits_f64(__builtin_isnan(v.f) ? (mc_f64_bits(v.f) | 0x0008000000000000ull) : 0xFFF8000000000000ull);
  }
  return mc_num_to_bits(mc_num_cast(mc_num_f(q), L, d), d);
}

constexpr size_t SER_NO_NAN = ~(size_t)0;

template <int L>
MC_DEV void ser_nan_fix(const uint8_t *src, int a, uint8_t *dst, int d, size_t n, size_t from,
                        unsigned long long *lds) {
  const int ds = mc_itemsize(d), as = mc_itemsize(a);
  if (threadIdx.x == 0) *lds = ~0ull;
  __syncthreads();
  for (size_t b = from; b < n; b += blockDim.x) {
    const size_t i = b + threadIdx.x;
    if (i < n && ser_is_nan_bits(mc_to_storage(mc_load_elem_u(dst, i, ds), d), d)) atomicMin(lds, (unsigned long long)i);
    __syncthreads();
    const unsigned long long k = *lds;
    __syncthreads();
    if (k != ~0ull) break;
  }
  const unsigned long long k0 = *lds;
  if (k0 >= n) return;
  const uint64_t v = ser_nan_tail_bits<L>(mc_load_elem_u(src, (size_t)k0, as), a, d);
  for (size_t i = (k0 == 0 ? 1 : (size_t)k0) + threadIdx.x; i < n; i += blockDim.x) mc_store_elem_u(dst, i, ds, v);
}

// G chain values as 16-B LDS accesses (p 16-B aligned)
template <typename T, int SER_G>
MC_DEV void ser_ld(const T *p, T (&r)[SER_G]) {
  typedef T vec __attribute__((ext_vector_type(16 / sizeof(T))));
  constexpr int W = 16 / sizeof(T);
#pragma unroll
  for (int v = 0; v < SER_G / W; ++v) {
    const vec x = reinterpret_cast<const vec *>(p)[v];
#pragma unroll
    for (int e = 0; e < W; ++e) r[v * W + e] = x[e];
  }
}
template <typename T, int SER_G>
MC_DEV void ser_st(T *p, const T (&r)[SER_G]) {
  typedef T vec __attribute__((ext_vector_type(16 / sizeof(T))));
  constexpr int W = 16 / sizeof(T);
#pragma unroll
  for (int v = 0; v < SER_G / W; ++v) {
    vec x;
#pragma unroll
    for (int e = 0; e < W; ++e) x[e] = r[v * W + e];
    reinterpret_cast<vec *>(p)[v] = x;
  }
}

// numpy's loop dtype of cumsum(enc: a, out=dec: d) for a float d:
// np.promote_types(a, d) (pinned against numpy for every pair by
// tests/test_gpu_delta_spec2.py): the wider float; an integer promotes to the
// smallest float that holds it (1-byte -> f2, 2-byte -> f4, wider -> f8)
static inline int mc_float_loop_dtype(int a, int d) {
  auto rank = [](int t) { return t == MC_F8 ? 3 : t == MC_F4 ? 2 : t == MC_F2 ? 1 : 0; };
  a = mc_dt_base(a);
  d = mc_dt_base(d);
  int fa;
  if (mc_is_float(a)) fa = a;
  else if (a == MC_B1 || mc_itemsize(a) == 1) fa = MC_F2;
  else if (mc_itemsize(a) == 2) fa = MC_F4;
  else fa = MC_F8;
  return rank(fa) > rank(d) ? fa : d;
}

// the speculative path's tile: FS_Q 16-B vectors per thread of W elements
constexpr int FS_Q = 4;
MC_HD constexpr int fs_w_of(int d) { return d == MC_F8 ? 2 : (d == MC_F4 ? 4 : 8); }
MC_HD constexpr size_t fs_tile_of(int d) { return (size_t)fs_w_of(d) * FS_Q * MC_BLOCK; }

static inline size_t fspec_ntiles(size_t n, int dt) {
  const size_t te = fs_tile_of(mc_dt_base(dt));
  return (n + te - 1) / te;
}

// the speculative decode serves any float dtype D with any numeric astype
// except bool whose loop dtype is D (casts as numpy's cumsum(enc, out=dec)
// does); a wider loop dtype (f8 astype into f4, ...) runs the serial chain
static inline bool fspec_types_ok(int astype, int dtype) {
  // the fix-up restarts from dtype values, so the loop dtype must be dtype
  return mc_is_float(dtype) && mc_valid_dtype(astype) && astype != MC_B1 &&
         mc_float_loop_dtype(astype, dtype) == mc_dt_base(dtype);
}

// tile totals, tile prefixes, per-tile first failures, the first failure
// (the last word, read by the tests)
static inline size_t fspec_ws_bytes(size_t n, int dt) { return (3 * fspec_ntiles(n, dt) + 1) * sizeof(uint64_t); }

// speculative float Delta decode of one chunk (workspace fspec_ws_bytes) /
// of `g` rows (fail: one word per row), output dtype f2 / f4 / f8, any
// astype whose loop dtype is the output dtype (mc_fspec_f*.hip); the _be_
// twins take a big-endian astype `a` and/or output (swo)
#define MC_FSPEC_DECL(T)                                                                                          \
  void mc_fspec_launch_##T(const uint8_t *s, uint8_t *d, size_t n, int a, void *ws, uint32_t *ticket,          \
                           hipStream_t st);                                                                    \
  void mc_fspec_rows_launch_##T(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a,           \
                                uint64_t *fail, unsigned g, hipStream_t st);                                   \
  void mc_fspec_launch_be_##T(const uint8_t *s, uint8_t *d, size_t n, int a, bool swo, void *ws,                 \
                              uint32_t *ticket, hipStream_t st);                                               \
  void mc_fspec_rows_launch_be_##T(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a,        \
                                   bool swo, uint64_t *fail, unsigned g, hipStream_t st);
MC_FSPEC_DECL(f2)
MC_FSPEC_DECL(f4)
MC_FSPEC_DECL(f8)
#undef MC_FSPEC_DECL

// numpy's serial float chain over `rows` chunks of n elements (astype a, may
// be big-endian; float dtype dt, may be big-endian); variant 0 = default
// schedule (mc_scan_serial.hip)
void mc_launch_serial_any(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n, size_t rows, int a, int dt,
                          hipStream_t st, int variant = 0);
