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
    for (int k = 0; k < 4; ++k) o[k] = (uint64_t)mc_wrap((int64_t)mc_scan_combine<OR_OP>(pre, p[k]), d);
    if (VEC && cnt == 4) {
      mc_store4(dst + i0 * ds, ds, o);
    } else {
      for (int k = 0; k < cnt; ++k) mc_store_elem_u(dst, i0 + k, ds, o[k]);
    }
    carry = mc_scan_combine<OR_OP>(carry, tot);
  }
}

// ---------------------------------------------------------------------------
// float dtypes: exact left-to-right accumulation, one workgroup per chunk.
// numpy's add.accumulate rounds after every add in order, so the adds form
// one dependent chain per chunk.  Two waves: lane 0 of wave 0 runs the chain
// over a block held in LDS (8 values per ds_read/ds_write group, only the add
// itself on the critical path) while wave 1 stores the previous block's
// results and loads + converts the next one into the other LDS slot with
// coalesced vector accesses, so HBM latency and the dtype conversions hide
// behind the chain.  A batch of chunks runs one chain per workgroup.
// ---------------------------------------------------------------------------
template <int D> struct SerAcc { using T = float; };
template <> struct SerAcc<MC_F8> { using T = double; };

template <int D>
MC_DEV typename SerAcc<D>::T ser_add(typename SerAcc<D>::T a, typename SerAcc<D>::T b) {
  if constexpr (D == MC_F2) {
    // numpy's half loop: float32 add, then npy_float_to_half.  The hardware
    // RNE conversion (denormals kept) gives the same half for every non-NaN
    // sum; NaN sums take numpy's payload-preserving routine.
    const float r = a + b;
    if (__builtin_isnan(r)) return mc_half_to_float(mc_float_to_half(r));
    return (float)(_Float16)r;
  } else {
    return a + b;
  }
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

constexpr int SER_UN = 8;              // vectors of 4 elements in flight per lane

// L: numpy's loop dtype for cumsum(enc: A, out=dec: D) is
// np.promote_types(A, D) (mc_float_loop_dtype): the running sum is kept in L
// and each result is cast to D on output (f8 input into f4 output
// accumulates in f8; f2 output of f4 input accumulates in f4).  The fix-up
// mode (startp) reads its carry back from dst, so it needs L == D.
template <int A_, int D, bool VEC, int SER_SLOT_BYTES = 32768, int SER_G = 16, int L = D>
__global__ __launch_bounds__(128) void k_scan_serial(const uint8_t *__restrict__ src,
                                                     size_t src_stride,
                                                     uint8_t *__restrict__ dst,
                                                     size_t dst_stride, size_t n, int a_rt,
                                                     const uint64_t *__restrict__ startp = nullptr) {
  static_assert(L == D || L == MC_F4 || L == MC_F8, "loop dtype");
  using T = typename SerAcc<L>::T;
  constexpr int BLK = SER_SLOT_BYTES / (int)sizeof(T);
  constexpr int DS = D == MC_F8 ? 8 : (D == MC_F4 ? 4 : 2);
  __shared__ __attribute__((aligned(16))) T slot[2][BLK + 2 * SER_G];
  const int a = A_ >= 0 ? A_ : a_rt;
  const int as = mc_itemsize(a);
  src += (size_t)blockIdx.x * src_stride;
  dst += (size_t)blockIdx.x * dst_stride;
  // fix-up mode (after k_fspec_apply / k_fspec_rows; startp[row]): the chain restarts at
  // the first element whose speculative value failed verification (rounded
  // down to a 128-B boundary so vector accesses stay aligned), carrying the
  // verified value before it; nothing to do if every element verified
  bool has_carry = false;
  T carry = 0;
  if (L == D && startp) {
    size_t s0 = (size_t)startp[blockIdx.x];
    if (s0 >= n) return;
    // restart on a 128-B line of dst: the chain's block loads/stores stay
    // line-aligned (a 16-B offset cost 15 % on 2048 x 1 MiB f4 rows)
    s0 &= ~(size_t)(128 / DS - 1);
    if (s0 > 0) {
      has_carry = true;
      const uint64_t cb = mc_load_elem_u(dst, s0 - 1, DS);
      if constexpr (D == MC_F8) carry = __builtin_bit_cast(double, cb);
      else if constexpr (D == MC_F4) carry = __builtin_bit_cast(float, (uint32_t)cb);
      else carry = (T)mc_num_from_bits(cb, D).f;
    }
    src += s0 * as;
    dst += s0 * DS;
    n -= s0;
  }
  const int lane = threadIdx.x & 63;
  const bool io = threadIdx.x >= 64;
  const size_t nb = (n + BLK - 1) / BLK;

  auto to_acc = [&](uint64_t bits) -> T {
    return (T)mc_num_cast(mc_num_from_bits(bits, a), a, L).f;
  };
  auto load_blk = [&](size_t b) {  // wave 1: src block b -> slot[b & 1]
    const size_t b0 = b * BLK;
    const int cnt = (int)min((size_t)BLK, n - b0);
    T *p = slot[b & 1];
    for (int r0 = 0; r0 < cnt; r0 += 4 * 64 * SER_UN) {
      uint64_t e[SER_UN][4];
#pragma unroll
      for (int u = 0; u < SER_UN; ++u) {
        const int j = r0 + 4 * (u * 64 + lane);
        if (VEC && j + 4 <= cnt) {
          mc_load4(src + (b0 + j) * as, as, e[u]);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            e[u][k] = j + k < cnt ? mc_load_elem_u(src, b0 + j + k, as) : 0;
        }
      }
#pragma unroll
      for (int u = 0; u < SER_UN; ++u) {
        const int j = r0 + 4 * (u * 64 + lane);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (j + k < cnt) p[j + k] = to_acc(e[u][k]);
      }
    }
  };
  auto store_blk = [&](size_t b) {  // wave 1: slot[b & 1] -> dst block b
    const size_t b0 = b * BLK;
    const int cnt = (int)min((size_t)BLK, n - b0);
    const T *p = slot[b & 1];
    for (int j = 4 * lane; j < cnt; j += 4 * 64) {
      uint64_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = j + k < cnt ? (L == D ? mc_num_to_bits(mc_num_f((double)p[j + k]), D)
                                     : mc_num_to_bits(mc_num_cast(mc_num_f((double)p[j + k]), L, D), D))
                           : 0;
      if (VEC && j + 4 <= cnt) {
        mc_store4(dst + (b0 + j) * DS, DS, o);
      } else {
        for (int k = 0; k < 4 && j + k < cnt; ++k) mc_store_elem_u(dst, b0 + j + k, DS, o[k]);
      }
    }
  };

  if (io) load_blk(0);
  __syncthreads();
  T acc = 0;
  for (size_t b = 0; b < nb; ++b) {
    if (io) {
      if (b >= 1) store_blk(b - 1);
      if (b + 1 < nb) load_blk(b + 1);
    } else if (lane == 0) {
      // software-pipelined chain: group g+1's LDS reads are in flight while
      // group g's adds run (ds_read latency ~50 cycles vs ~G dependent adds)
      T *p = slot[b & 1];
      const int cnt = (int)min((size_t)BLK, n - b * BLK);
      int j = 0;
      if (b == 0) {  // out[0] = x[0] exactly (no add), then align to a group
        acc = has_carry ? ser_add<L>(carry, p[0]) : p[0];
        p[0] = acc;
        const int m = cnt < SER_G ? cnt : SER_G;
        for (int k = 1; k < m; ++k) {
          acc = ser_add<L>(acc, p[k]);
          p[k] = acc;
        }
        j = m;
      }
      // two register groups alternate: while one group's adds run, the other
      // group's 16-B LDS reads are in flight (the slot is padded by 2 groups,
      // so the read-ahead never leaves it)
      if (j + 2 * SER_G <= cnt) {
        T ga[SER_G], gb[SER_G];
        ser_ld<T, SER_G>(p + j, ga);
        for (; j + 2 * SER_G <= cnt; j += 2 * SER_G) {
          ser_ld<T, SER_G>(p + j + SER_G, gb);
          __builtin_amdgcn_sched_barrier(0);  // keep the read-ahead ahead of the adds
#pragma unroll
          for (int k = 0; k < SER_G; ++k) {
            acc = ser_add<L>(acc, ga[k]);
            ga[k] = acc;
          }
          ser_st<T, SER_G>(p + j, ga);
          ser_ld<T, SER_G>(p + j + 2 * SER_G, ga);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < SER_G; ++k) {
            acc = ser_add<L>(acc, gb[k]);
            gb[k] = acc;
          }
          ser_st<T, SER_G>(p + j + SER_G, gb);
        }
      }
      for (; j < cnt; ++j) {
        acc = ser_add<L>(acc, p[j]);
        p[j] = acc;
      }
    }
    __syncthreads();
  }
  if (io) store_blk(nb - 1);
}

// (slot bytes, group) per schedule: a 32 KiB slot amortises the block
// barrier for one long chain; a batch needs small slots so that many chains
// (workgroups) fit a CU's LDS at once (2 x 32 KiB slots allow only 2).
// numpy's loop dtype of cumsum(enc: a, out=dec: d) for a float d:
// np.promote_types(a, d) (pinned against numpy for every pair by
// tests/test_gpu_delta_spec2.py): the wider float; an integer promotes to the
// smallest float that holds it (1-byte -> f2, 2-byte -> f4, wider -> f8)
static int mc_float_loop_dtype(int a, int d) {
  auto rank = [](int t) { return t == MC_F8 ? 3 : t == MC_F4 ? 2 : t == MC_F2 ? 1 : 0; };
  int fa;
  if (mc_is_float(a)) fa = a;
  else if (a == MC_B1 || mc_itemsize(a) == 1) fa = MC_F2;
  else if (mc_itemsize(a) == 2) fa = MC_F4;
  else fa = MC_F8;
  return rank(fa) > rank(d) ? fa : d;
}

template <int D>
static void launch_serial(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n,
                          size_t rows, int a, hipStream_t st, int variant = 0) {
  const int as = mc_itemsize(a);
  const int loop = mc_float_loop_dtype(a, D);
  if (loop != D) {  // accumulate in the wider loop dtype, cast each result to D
    const bool v = ((uintptr_t)s % (4 * as) == 0) && (ss % (4 * as) == 0) &&
                   ((uintptr_t)d % (4 * mc_itemsize(D)) == 0) && (dss % (4 * mc_itemsize(D)) == 0);
    const unsigned g = (unsigned)rows;
    if constexpr (D != MC_F8) {
      if (loop == MC_F8) {
        if (v) k_scan_serial<-1, D, true, 8192, 16, MC_F8><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
        else k_scan_serial<-1, D, false, 8192, 16, MC_F8><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
        return;
      }
    }
    if constexpr (D == MC_F2) {
      if (v) k_scan_serial<-1, D, true, 8192, 16, MC_F4><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
      else k_scan_serial<-1, D, false, 8192, 16, MC_F4><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
    }
    return;
  }
  const bool vec = ((uintptr_t)s % (4 * as) == 0) && (ss % (4 * as) == 0) &&
                   ((uintptr_t)d % (4 * mc_itemsize(D)) == 0) && (dss % (4 * mc_itemsize(D)) == 0);
  // measured (tools/probe_delta.py, profiles/r01/probe_delta.json): one chain
  // 32 KiB / 32; 2048 chains of 1 MiB 8 KiB slots, 32-value groups for f4
  // and 16 for f8
  if (variant == 0) variant = rows >= 256 ? (D == MC_F8 ? 3 : 4) : 2;
  const unsigned g = (unsigned)rows;
  if (vec && a == D) {
    switch (variant) {
      case 1: k_scan_serial<D, D, true, 32768, 16><<<g, 128, 0, st>>>(s, ss, d, dss, n, a); break;
      case 2: k_scan_serial<D, D, true, 32768, 32><<<g, 128, 0, st>>>(s, ss, d, dss, n, a); break;
      case 3: k_scan_serial<D, D, true, 8192, 16><<<g, 128, 0, st>>>(s, ss, d, dss, n, a); break;
      case 4: k_scan_serial<D, D, true, 8192, 32><<<g, 128, 0, st>>>(s, ss, d, dss, n, a); break;
      default: k_scan_serial<D, D, true, 4096, 32><<<g, 128, 0, st>>>(s, ss, d, dss, n, a); break;
    }
  } else if (vec) {
    k_scan_serial<-1, D, true, 8192, 16><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
  } else {
    k_scan_serial<-1, D, false, 8192, 16><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
  }
}

static void launch_serial_any(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n,
                              size_t rows, int a, int dt, hipStream_t st, int variant = 0) {
  if (dt == MC_F8) launch_serial<MC_F8>(s, ss, d, dss, n, rows, a, st, variant);
  else if (dt == MC_F4) launch_serial<MC_F4>(s, ss, d, dss, n, rows, a, st, variant);
  else launch_serial<MC_F2>(s, ss, d, dss, n, rows, a, st, variant);
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
        o[k] = (uint64_t)mc_wrap((int64_t)mc_scan_combine<OR_OP>(pre, p[k]), d);
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
template <int ES, bool NT = true>
MC_DEV void ds_load_half(const uint8_t *src, size_t n, size_t e0, dacc_t<ES> (&v)[ds_per<ES>()], int at) {
  constexpr int H = ds_per<ES>() / 2;
  if (e0 + H <= n) {
    const mc_u32x4 w = mc_ld16<NT>(src + e0 * ES);
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
    for (int i = 0; i < H; ++i) v[at + i] = e0 + i < n ? (dacc_t<ES>)mc_load_elem(src, e0 + i, ES) : 0;
  }
}


template <int ES>
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
      const mc_u32x4 w0 = mc_ld16<true>(tb + 16 * (size_t)threadIdx.x);
      const mc_u32x4 w1 = mc_ld16<true>(tb + 16 * (size_t)(MC_BLOCK + threadIdx.x));
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
      ds_load_half<ES>(src, n, tb + (size_t)threadIdx.x * HALF, v[h], 0);
      ds_load_half<ES>(src, n, tb + (size_t)(MC_BLOCK + threadIdx.x) * HALF, v[h], HALF);
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
template <int ES>
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
    mc_st16<true>(dst + e0 * ES, mc_u32x4{d[0], d[1], d[2], d[3]});
  } else {
    for (int i = 0; i < H && e0 + i < n; ++i) mc_store_elem(dst, e0 + i, ES, (uint64_t)v[at + i]);
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
template <int ES>
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
  ds_load_half<ES>(src, n, ea0, v, 0);
  ds_load_half<ES>(src, n, eb0, v, H);
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
  ds_store_half<ES>(dst, n, ea0, v, 0);
  ds_store_half<ES>(dst, n, eb0, v, H);
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
template <int ES>
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
  ds_load_half<ES>(src, n, oa, nxt, 0);
  ds_load_half<ES>(src, n, ob, nxt, H);
  int parity = 0;
  for (size_t base = 0; base < n; base += TE, parity ^= 1) {
    T v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = nxt[i];
    if (base + TE < n) {
      ds_load_half<ES>(src, n, base + TE + oa, nxt, 0);
      ds_load_half<ES>(src, n, base + TE + ob, nxt, H);
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
    ds_store_half<ES>(dst, n, base + oa, v, 0);
    ds_store_half<ES>(dst, n, base + ob, v, H);
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

template <int ES, bool NT = false>
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
      const mc_u32x4 w0 = mc_ld16<NT>(tb + 16 * (size_t)threadIdx.x);
      const mc_u32x4 w1 = mc_ld16<NT>(tb + 16 * (size_t)(MC_BLOCK + threadIdx.x));
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
      ds_load_half<ES, NT>(src, n, tb + (size_t)threadIdx.x * HALF, v[h], 0);
      ds_load_half<ES, NT>(src, n, tb + (size_t)(MC_BLOCK + threadIdx.x) * HALF, v[h], HALF);
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

template <int ES, bool NT = false>
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
  uint32_t x = (wave == 0 && (size_t)lane < g) ? gtot[lane] : 0u;  // before the data loads
  for (unsigned j = threadIdx.x; j < GT && gt0 + j < tile; j += MC_BLOCK) x += tile_tot[gt0 + j];
  const size_t ea0 = tile * ds_tile<ES>() + (size_t)threadIdx.x * H;
  const size_t eb0 = tile * ds_tile<ES>() + (size_t)(MC_BLOCK + threadIdx.x) * H;
  T v[PER];
  ds_load_half<ES, NT>(src, n, ea0, v, 0);
  ds_load_half<ES, NT>(src, n, eb0, v, H);
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
  ds_store_half<ES>(dst, n, ea0, v, 0);
  ds_store_half<ES>(dst, n, eb0, v, H);
}

template <int ES>
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
  if (ntm & 1) k_dscan_reduce_g<ES, true><<<rg, MC_BLOCK, 0, st>>>(s, n, ws, ticket, ntiles, gt);
  else k_dscan_reduce_g<ES, false><<<rg, MC_BLOCK, 0, st>>>(s, n, ws, ticket, ntiles, gt);
  if (ntm & 2) k_dscan_apply_g<ES, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, ws, ntiles, gt);
  else k_dscan_apply_g<ES, false><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, ws, ntiles, gt);
}

// mc_sched.dscan = 0 selects the generic three-pass kernels (lab A/B only)
static bool dscan_enabled() { return mc_sched.dscan != 0; }

template <int ES>
static void launch_dscan(const uint8_t *s, uint8_t *d, size_t n, uint64_t *ws, hipStream_t st) {
  const size_t ntiles = (n + ds_tile<ES>() - 1) / ds_tile<ES>();
  const size_t ngroups = (ntiles + DS_GROUP - 1) / DS_GROUP;
  uint64_t *group = ws, *part = ws + ngroups, *gpre = part + DS_GROUP * ngroups;
  k_dscan_reduce<ES><<<(unsigned)ngroups, MC_BLOCK, 0, st>>>(s, n, group, part);
  mc_launch_scan_sums_mw<false>(group, gpre, ngroups, st);
  k_dscan_apply<ES><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, gpre, part);
}


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
template <int D> struct FsStore { using S = float; using V = float; };
template <> struct FsStore<MC_F8> { using S = double; using V = double; };
template <> struct FsStore<MC_F2> { using S = _Float16; using V = float; };

template <int A_, int D>
struct FsT {
  using S = typename FsStore<D>::S;  // stored element
  using V = typename FsStore<D>::V;  // arithmetic value (numpy's loop type)
  static constexpr int W = 16 / (int)sizeof(S);
  typedef S svec __attribute__((ext_vector_type(W)));
  MC_DEV static V from_bits(uint64_t bits, int a) {  // enc element -> its D value
    return (V)mc_num_cast(mc_num_from_bits(bits, a), a, D).f;
  }
  MC_DEV static S round(double x) { return (S)x; }  // candidate (any rounding)
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

constexpr int FS_Q = 4;
MC_HD constexpr int fs_w_of(int d) { return d == MC_F8 ? 2 : (d == MC_F4 ? 4 : 8); }
MC_HD constexpr size_t fs_tile_of(int d) { return (size_t)fs_w_of(d) * FS_Q * MC_BLOCK; }
template <int D> constexpr size_t fs_tile() { return fs_tile_of(D); }

template <int D>
MC_DEV size_t fs_elem0(size_t t0, int q) {  // first element of this thread's vector in segment q
  return t0 + (size_t)q * fs_w_of(D) * MC_BLOCK + (size_t)threadIdx.x * fs_w_of(D);
}

template <int A_, int D>
MC_DEV void fs_load(const uint8_t *src, size_t n, size_t t0, int a,
                    typename FsT<A_, D>::V (&v)[FS_Q][FsT<A_, D>::W]) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
  if constexpr (A_ == D) {
    // default-policy loads: the apply pass re-reads what the reduce pass read
    // and finds part of it in the Infinity Cache (256 MiB f4 smooth decode
    // 158-162 -> 154 us against nontemporal loads; f8 unchanged)
#pragma unroll
    for (int q = 0; q < FS_Q; ++q) {
      const size_t e0 = fs_elem0<D>(t0, q);
      if (e0 + W <= n) {
        const typename Tr::svec x =
            *reinterpret_cast<const typename Tr::svec *>(src + e0 * sizeof(typename Tr::S));
#pragma unroll
        for (int e = 0; e < W; ++e) v[q][e] = (typename Tr::V)x[e];
      } else {
#pragma unroll
        for (int e = 0; e < W; ++e)
          v[q][e] = e0 + e < n ? (typename Tr::V)reinterpret_cast<const typename Tr::S *>(src)[e0 + e]
                               : (typename Tr::V)0;
      }
    }
  } else if constexpr (A_ == MC_F4 && D == MC_F8) {
    // f8 <- f4 (the dispatch checks 8-B alignment): one 8-B load of the
    // thread's 2 float32 per vector, the casts in registers.  The components
    // are copied out before the bit casts: __builtin_bit_cast of an
    // ext_vector component reads component 0 (seen in the gfx950 assembly)
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

template <int A_, int D>
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
      __builtin_nontemporal_store(x, reinterpret_cast<typename Tr::svec *>(dst + e0 * sizeof(typename Tr::S)));
    } else {
      for (int e = 0; e < W && e0 + e < n; ++e) reinterpret_cast<typename Tr::S *>(dst)[e0 + e] = c[q][e];
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

template <typename V, int W>
MC_DEV void fs_tile_scan(const V (&v)[FS_Q][W], double (&p)[FS_Q][W], double (&lds)[FS_Q][MC_BLOCK / 64]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double incl[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    p[q][0] = (double)v[q][0];
#pragma unroll
    for (int e = 1; e < W; ++e) p[q][e] = p[q][e - 1] + (double)v[q][e];
    incl[q] = p[q][W - 1];
  }
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) incl[q] = mc_wave_scan_f64(incl[q]);
  double ex[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    if (lane == 63) lds[q][wave] = incl[q];
    ex[q] = mc_wave_shr1_f64(incl[q]);
  }
  __syncthreads();
  double base = 0.0;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    double w = 0.0, tot = 0.0;
#pragma unroll
    for (int j = 0; j < MC_BLOCK / 64; ++j) {
      if (j < wave) w = w + lds[q][j];
      tot = tot + lds[q][j];
    }
    const double pre = base + (lane ? w + ex[q] : w);
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

template <int A_, int D>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_reduce(const uint8_t *__restrict__ src, size_t n, int a,
                                                          double *__restrict__ sums) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
  __shared__ double lds[FS_Q][MC_BLOCK / 64];
  typename Tr::V v[FS_Q][W];
  fs_load<A_, D>(src, n, (size_t)blockIdx.x * fs_tile<D>(), a, v);
  double p[FS_Q][W];
  fs_tile_scan<typename Tr::V, W>(v, p, lds);
  if (threadIdx.x == MC_BLOCK - 1) sums[blockIdx.x] = p[FS_Q - 1][W - 1];
}

template <int A_, int D>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_apply(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t n, int a,
                                                         const double *__restrict__ sums,
                                                         const double *__restrict__ pre_t,
                                                         uint64_t *__restrict__ tfail,
                                                         uint64_t *__restrict__ fail) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  constexpr int W = Tr::W;
  __shared__ double lds[FS_Q][MC_BLOCK / 64];
  __shared__ S ldsc[FS_Q][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t tile = blockIdx.x;
  const size_t t0 = tile * fs_tile<D>();
  // every tile is verified and stored, also past an earlier failure: the
  // walker (k_fspec_walk) re-bases at the first failing element and jumps
  // over the tiles recorded here as verified once it is back in sync
  typename Tr::V v[FS_Q][W];
  fs_load<A_, D>(src, n, t0, a, v);
  double p[FS_Q][W];
  fs_tile_scan<typename Tr::V, W>(v, p, lds);
  const double Sp = pre_t[tile];  // the tile's prefix
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
  const S pbound = tile ? Tr::round(pre_t[tile - 1] + sums[tile - 1]) : (S)0;
  S p0[FS_Q];
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    if (lane) p0[q] = up[q];
    else if (wave) p0[q] = ldsc[q][wave - 1];
    else p0[q] = q ? ldsc[q - 1][MC_BLOCK / 64 - 1] : pbound;
  }
  uint64_t first = fs_check<A_, D>(c, v, p0, t0, n);
  fs_store<A_, D>(dst, n, t0, c);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(first, off, 64);
    first = o < first ? o : first;
  }
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
template <int A_, int D>
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_rows(const uint8_t *__restrict__ src,
                                                        size_t src_stride, uint8_t *__restrict__ dst,
                                                        size_t dst_stride, size_t n, int a,
                                                        uint64_t *__restrict__ fail) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  constexpr int W = Tr::W;
  __shared__ double lds[2][FS_Q][MC_BLOCK / 64];
  __shared__ S ldsc[2][FS_Q][MC_BLOCK / 64];
  __shared__ uint64_t ldsf[2][MC_BLOCK / 64];
  __shared__ double ldsp[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  src += (size_t)blockIdx.x * src_stride;
  dst += (size_t)blockIdx.x * dst_stride;
  double carry = 0.0;
  S prevc = (S)0;
  int par = 0;
  typename Tr::V nv[FS_Q][W];
  fs_load<A_, D>(src, n, 0, a, nv);
  for (size_t t0 = 0; t0 < n; t0 += fs_tile<D>(), par ^= 1) {
    typename Tr::V v[FS_Q][W];
#pragma unroll
    for (int q = 0; q < FS_Q; ++q)
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = nv[q][e];
    if (t0 + fs_tile<D>() < n) fs_load<A_, D>(src, n, t0 + fs_tile<D>(), a, nv);  // next tile in flight
    double p[FS_Q][W];
    fs_tile_scan<typename Tr::V, W>(v, p, lds[par]);
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
    uint64_t first = fs_check<A_, D>(c, v, p0, t0, n);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t o = __shfl_xor(first, off, 64);
      first = o < first ? o : first;
    }
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
    fs_store<A_, D>(dst, n, t0, c);
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

// The serial chain over p[j..cnt) in place (acc = the value before p[j]),
// numpy's order: two read groups alternate so the next group's LDS reads are
// in flight while the current group's adds run (as in k_scan_serial).  p is
// padded by 2 groups past cnt.
template <int D>
MC_DEV typename SerAcc<D>::T fsw_chain(typename SerAcc<D>::T *p, int j, int cnt, typename SerAcc<D>::T acc) {
  using T = typename SerAcc<D>::T;
  for (; j < cnt && (j & (FSW_G - 1)); ++j) {
    acc = ser_add<D>(acc, p[j]);
    p[j] = acc;
  }
  if (j + 2 * FSW_G <= cnt) {
    T ga[FSW_G], gb[FSW_G];
    ser_ld<T, FSW_G>(p + j, ga);
    for (; j + 2 * FSW_G <= cnt; j += 2 * FSW_G) {
      ser_ld<T, FSW_G>(p + j + FSW_G, gb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < FSW_G; ++k) {
        acc = ser_add<D>(acc, ga[k]);
        ga[k] = acc;
      }
      ser_st<T, FSW_G>(p + j, ga);
      ser_ld<T, FSW_G>(p + j + 2 * FSW_G, ga);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < FSW_G; ++k) {
        acc = ser_add<D>(acc, gb[k]);
        gb[k] = acc;
      }
      ser_st<T, FSW_G>(p + j + FSW_G, gb);
    }
  }
  for (; j < cnt; ++j) {
    acc = ser_add<D>(acc, p[j]);
    p[j] = acc;
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

template <int A_, int D>
MC_DEV void fsw_load(const uint8_t *src, size_t n, size_t t0, int a,
                     typename FsT<A_, D>::V (&v)[FS_Q][FsT<A_, D>::W]) {
  using Tr = FsT<A_, D>;
  constexpr int W = Tr::W;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    const size_t e0 = t0 + (size_t)fsw_li(q, 0, W);
    if constexpr (A_ == D) {
      if (e0 + W <= n) {
        const typename Tr::svec x =
            __builtin_nontemporal_load(reinterpret_cast<const typename Tr::svec *>(src + e0 * sizeof(typename Tr::S)));
#pragma unroll
        for (int e = 0; e < W; ++e) v[q][e] = (typename Tr::V)x[e];
      } else {
#pragma unroll
        for (int e = 0; e < W; ++e)
          v[q][e] = e0 + e < n ? (typename Tr::V)reinterpret_cast<const typename Tr::S *>(src)[e0 + e]
                               : (typename Tr::V)0;
      }
    } else {
      const int as = mc_itemsize(a);
      uint64_t b[W];
#pragma unroll
      for (int e = 0; e < W; ++e) b[e] = e0 + e < n ? mc_load_elem_u(src, e0 + e, as) : 0;
#pragma unroll
      for (int e = 0; e < W; ++e) v[q][e] = e0 + e < n ? Tr::from_bits(b[e], a) : (typename Tr::V)0;
    }
  }
}

template <int A_, int D>
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
      __builtin_nontemporal_store(x, reinterpret_cast<typename Tr::svec *>(dst + e0 * sizeof(typename Tr::S)));
    } else {
      for (int e = 0; e < W && e0 + e < n; ++e) reinterpret_cast<typename Tr::S *>(dst)[e0 + e] = c[q][e];
    }
  }
}

// p[q][e] = the tile-relative inclusive double prefix of this thread's
// elements in the walker layout (any fixed association: candidates only
// propose, the per-element check decides)
template <typename V, int W>
MC_DEV void fsw_scan(const V (&v)[FS_Q][W], double (&p)[FS_Q][W], double *ldsq) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double base = 0.0;
#pragma unroll
  for (int q = 0; q < FS_Q; ++q) {
    p[q][0] = (double)v[q][0];
#pragma unroll
    for (int e = 1; e < W; ++e) p[q][e] = p[q][e - 1] + (double)v[q][e];
    const double incl = mc_wave_scan_f64(p[q][W - 1]);
    const double ex = mc_wave_shr1_f64(incl);
    const double pre = base + (lane ? ex : 0.0);
#pragma unroll
    for (int e = 0; e < W; ++e) p[q][e] = pre + p[q][e];
    base = base + fsw_readlane(incl, 63);
  }
  if (lane == 0) ldsq[wave] = base;  // the quarter's total
  __syncthreads();
  double off = 0.0;
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
template <int A_, int D>
MC_DEV typename FsT<A_, D>::S fsw_stream(const uint8_t *src, uint8_t *dst, size_t n, int a, size_t tb, size_t te,
                                         typename FsT<A_, D>::S yin, bool has_in,
                                         typename FsT<A_, D>::V (*xs)[fs_tile_of(D) + 2 * FSW_G],
                                         typename FsT<A_, D>::S *ldsy) {
  using Tr = FsT<A_, D>;
  using S = typename Tr::S;
  using V = typename Tr::V;
  constexpr int W = Tr::W;
  constexpr int TE = (int)fs_tile<D>();
  constexpr int NV = TE / W;  // vectors per tile
  const int wave = threadIdx.x >> 6;
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
          if (k < NV && e0 + W <= n)
            xv[u] = __builtin_nontemporal_load(reinterpret_cast<const typename Tr::svec *>(src + e0 * sizeof(S)));
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
        __builtin_nontemporal_store(x, reinterpret_cast<typename Tr::svec *>(dst + e0 * sizeof(S)));
      } else {
        for (int e = 0; e < W && e0 + e < n; ++e) reinterpret_cast<S *>(dst)[e0 + e] = Tr::store(buf[k * W + e]);
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
        if (t0 == 0 && !has_in) {  // the chunk's first element: out[0] = enc[0]
          acc = p[0];
          j = 1;
        }
        acc = fsw_chain<D>(p, j, cnt, acc);
        if (t + 1 == te) *ldsy = Tr::store(acc);
      }
    } else {
      const int io = threadIdx.x - 64;
      if (t > tb) io_store(t - 1, xs[(t - 1) & 1], io, MC_BLOCK - 64);
      if (t + 1 < te) io_load(t + 1, xs[(t + 1) & 1], io, MC_BLOCK - 64);
    }
    __syncthreads();
  }
  io_store(te - 1, xs[(te - 1) & 1], threadIdx.x, MC_BLOCK);
  const S y = *ldsy;
  __syncthreads();  // the buffers and ldsy are free again
  return y;
}

template <int A_, int D>
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
  constexpr int W = Tr::W;
  constexpr int TE = (int)fs_tile<D>();
  constexpr int QE = fsw_qe<D>();
  constexpr int NOFAIL = 0x7fffffff;
  // per pass, each wave publishes its last candidate, its first element
  // (value, candidate, prefix) and its first failure inside the quarter
  __shared__ double ldsq[FSW_NW];
  __shared__ S lds_last[2][FSW_NW], lds_bc[2][FSW_NW], lds_fv[2][FSW_NW];
  __shared__ V lds_bv[2][FSW_NW];
  __shared__ double lds_bp[2][FSW_NW], lds_fp[2][FSW_NW];
  __shared__ int lds_fi[2][FSW_NW];
  __shared__ uint64_t ldsx[FSW_NW];
  __shared__ S ldsy;
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
  if (single) {
    const uint64_t f = *fail;  // the first index that failed at apply time
    if (f >= n) return;        // everything verified: dst is final
    t = (size_t)(f / TE);
    has_in = t > 0;
    if (has_in) yin = Tr::round(pre[t - 1] + sums[t - 1]);  // tile t-1 verified: its last candidate
  } else {
    // a row that k_fspec_rows left at its first failing tile (rowfail = its
    // start; n when the row verified): resume there from the last stored value
    const uint64_t f = rowfail[blockIdx.x];
    if (f >= n) return;
    t = (size_t)(f / TE);
    has_in = t > 0;
    if (has_in) yin = reinterpret_cast<const S *>(dst)[t * (size_t)TE - 1];
  }
  int serial_run = 0, par = 0;
  size_t next_probe = 0, gap = FSW_PROBE;  // serial tiles stream until next_probe
  V nv[FS_Q][W];
  fsw_load<A_, D>(src, n, t * TE, a, nv);
  while (t < ntiles) {
    if (serial_run > 0 && t < next_probe) {
      // noise-like stretch: serial streaming up to the next probe tile
      const size_t te = next_probe < ntiles ? next_probe : ntiles;
      yin = fsw_stream<A_, D>(src, dst, n, a, t, te, yin, has_in, xs2, &ldsy);
      has_in = true;
      serial_run += (int)(te - t);
      t = te;
      if (t >= ntiles) break;
      fsw_load<A_, D>(src, n, t * (size_t)TE, a, nv);
      if (single && Tr::bits(yin) == Tr::bits(Tr::round(pre[t - 1] + sums[t - 1]))) {
        const size_t nt = fsw_next_failed(tfail, t, ntiles, ldsx);
        if (nt >= ntiles) break;
        if (nt != t) {
          t = nt;
          yin = Tr::round(pre[nt - 1] + sums[nt - 1]);
          fsw_load<A_, D>(src, n, nt * (size_t)TE, a, nv);
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
    if (t + 1 < ntiles) fsw_load<A_, D>(src, n, t0 + TE, a, nv);  // the usual successor, in flight
    const int cnt = (int)(n - t0 < (size_t)TE ? n - t0 : (size_t)TE);
    const bool first_tile = t0 == 0;
    S c[FS_Q][W];
    int fpos = -1;  // elements at local index <= fpos are final
    S fixed = yin;  // the true value at fpos
    bool go_serial = false;
    const int cap = serial_run > 0 ? FSW_PROBE_CAP : FSW_CAP;
    if (!go_serial) {
      double p[FS_Q][W];
      fsw_scan<V, W>(v, p, ldsq);
      // candidates c_i = D(kb + p_i) with kb = y_base - p_base (one add per
      // element; any association proposes, the check decides)
      double kb = has_in ? (double)Tr::val(yin) : 0.0;
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
            const bool ok = (Tr::bits(c[q][e]) == Tr::bits(r)) & Tr::finite(c[q][e]);
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
        double wp = 0.0;
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
          double pk = 0.0;
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
        double fp = 0.0;
#pragma unroll
        for (int w = FSW_NW - 1; w >= 0; --w) {
          const int wfi = lds_fi[par][w];
          const S wfv = lds_fv[par][w], bc = lds_bc[par][w];
          const double wfp = lds_fp[par][w], bp = lds_bp[par][w];
          const V bv = lds_bv[par][w];
          const S pe = w ? lds_last[par][w - 1] : yin;  // w = 0: only checked while fpos < 0
          f = fsw_sel(wfi != NOFAIL, wfi, f);
          fv = fsw_sel(wfi != NOFAIL, wfv, fv);
          fp = fsw_sel(wfi != NOFAIL, wfp, fp);
          const int lb = w * QE;
          const S r = Tr::store((w == 0 && first_tile) ? bv : Tr::step(Tr::val(pe), bv));  // out[0] = enc[0]
          const bool bad = (lb > fpos) & (lb < cnt) & !((Tr::bits(bc) == Tr::bits(r)) & Tr::finite(bc));
          f = fsw_sel(bad, lb, f);
          fv = fsw_sel(bad, r, fv);
          fp = fsw_sel(bad, bp, fp);
        }
        if (f == NOFAIL) break;  // the tile verified from the true values before it
        // re-base at f: numpy's value there (its predecessor is verified)
        fpos = f;
        fixed = fv;
        kb = (double)Tr::val(fv) - fp;
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
    fsw_store<A_, D>(dst, n, t0, c);
    if (t + 1 >= ntiles) break;
    if (single && Tr::bits(yin) == Tr::bits(Tr::round(pre[t] + sums[t]))) {
      // in sync with the apply pass: tiles that verified there are final
      const size_t nt = fsw_next_failed(tfail, t + 1, ntiles, ldsx);
      if (nt >= ntiles) break;
      if (nt != t + 1) {
        t = nt;
        yin = Tr::round(pre[nt - 1] + sums[nt - 1]);
        fsw_load<A_, D>(src, n, nt * (size_t)TE, a, nv);
        continue;
      }
    }
    ++t;
  }
}

// mc_sched.fspec = 0 disables the speculative float path (lab A/B: serial only)
static bool fspec_enabled() { return mc_sched.fspec != 0; }

static size_t fspec_ntiles(size_t n, int dt) {
  const size_t te = fs_tile_of(dt);
  return (n + te - 1) / te;
}

// the speculative decode serves any float dtype D with any numeric astype
// except bool whose loop dtype is D (casts as numpy's cumsum(enc, out=dec)
// does); a wider loop dtype (f8 astype into f4, ...) runs the serial chain
static bool fspec_types_ok(int astype, int dtype) {
  // the fix-up restarts from dtype values, so the loop dtype must be dtype
  return mc_is_float(dtype) && mc_valid_dtype(astype) && astype != MC_B1 &&
         mc_float_loop_dtype(astype, dtype) == dtype;
}

// tile totals, tile prefixes, per-tile first failures, the first failure
// (the last word, read by the tests)
static size_t fspec_ws_bytes(size_t n, int dt) { return (3 * fspec_ntiles(n, dt) + 1) * sizeof(uint64_t); }

// Tile prefixes by many workgroups (one per 256 tiles): workgroup g sums
// all totals before its range itself (coalesced, 8 loads in flight per
// thread) and scans its own 256.  A one-workgroup scan (LDS-staged, 4096
// totals per round) was bound by a single CU's bandwidth: 14.7 us for
// 16 Ki tiles against 7.9 us here; reading the earlier totals redundantly
// spreads that over ntiles/256 CUs.  Any association is
// fine: the apply pass only relies on the stored pre[] and sums[].
__global__ __launch_bounds__(MC_BLOCK) void k_fspec_pre(const double *__restrict__ sums,
                                                       double *__restrict__ pre, size_t ntiles,
                                                       uint64_t *__restrict__ tfail,
                                                       uint64_t *__restrict__ fail, size_t n) {
  __shared__ double lds[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t b = (size_t)blockIdx.x * MC_BLOCK;
  double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  size_t i = threadIdx.x;
  for (; i + 7 * MC_BLOCK < b; i += 8 * MC_BLOCK) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += sums[i + (size_t)k * MC_BLOCK];
  }
  for (; i < b; i += MC_BLOCK) a[0] += sums[i];
  double acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
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

template <int A_, int D>
static void launch_fspec(const uint8_t *s, uint8_t *d, size_t n, int a, void *ws, hipStream_t st) {
  const size_t ntiles = fspec_ntiles(n, D);
  double *sums = static_cast<double *>(ws), *pre = sums + ntiles;
  uint64_t *tfail = reinterpret_cast<uint64_t *>(pre + ntiles), *fail = tfail + ntiles;
  k_fspec_reduce<A_, D><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, n, a, sums);
  k_fspec_pre<<<(unsigned)((ntiles + MC_BLOCK - 1) / MC_BLOCK), MC_BLOCK, 0, st>>>(sums, pre, ntiles, tfail, fail, n);
  k_fspec_apply<A_, D><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, a, sums, pre, tfail, fail);
  // one walker from the first failing tile (returns at once if none failed)
  k_fspec_walk<A_, D><<<1, MC_BLOCK, 0, st>>>(s, 0, d, 0, n, a, nullptr, sums, pre, tfail, fail);
}

static void launch_fspec_any(const uint8_t *s, uint8_t *d, size_t n, int a, int dt, void *ws, hipStream_t st) {
  if (dt == MC_F8) {
    if (a == MC_F8) launch_fspec<MC_F8, MC_F8>(s, d, n, a, ws, st);
    else if (a == MC_F4 && (uintptr_t)s % 8 == 0) launch_fspec<MC_F4, MC_F8>(s, d, n, a, ws, st);
    else launch_fspec<-1, MC_F8>(s, d, n, a, ws, st);
  } else if (dt == MC_F4) {
    if (a == MC_F4) launch_fspec<MC_F4, MC_F4>(s, d, n, a, ws, st);
    else launch_fspec<-1, MC_F4>(s, d, n, a, ws, st);
  } else {
    if (a == MC_F2) launch_fspec<MC_F2, MC_F2>(s, d, n, a, ws, st);
    else launch_fspec<-1, MC_F2>(s, d, n, a, ws, st);
  }
}

// the speculative rows pass, then one walker per row that failed (rows that
// verified return at once)
template <int A_, int D>
static void launch_fspec_rows(const uint8_t *sc, size_t src_stride, uint8_t *dc, size_t dst_stride, size_t n, int a,
                              uint64_t *fail, unsigned g, hipStream_t st) {
  k_fspec_rows<A_, D><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n, a, fail);
  k_fspec_walk<A_, D><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n, a, fail, nullptr, nullptr, nullptr,
                                            nullptr);
}

static void launch_fspec_rows_any(const uint8_t *sc, size_t ss, uint8_t *dc, size_t ds, size_t n, int a, int dt,
                                  uint64_t *fail, unsigned g, hipStream_t st) {
  if (dt == MC_F8) {
    if (a == MC_F8) launch_fspec_rows<MC_F8, MC_F8>(sc, ss, dc, ds, n, a, fail, g, st);
    else if (a == MC_F4 && (uintptr_t)sc % 8 == 0 && ss % 8 == 0)
      launch_fspec_rows<MC_F4, MC_F8>(sc, ss, dc, ds, n, a, fail, g, st);
    else launch_fspec_rows<-1, MC_F8>(sc, ss, dc, ds, n, a, fail, g, st);
  } else if (dt == MC_F4) {
    if (a == MC_F4) launch_fspec_rows<MC_F4, MC_F4>(sc, ss, dc, ds, n, a, fail, g, st);
    else launch_fspec_rows<-1, MC_F4>(sc, ss, dc, ds, n, a, fail, g, st);
  } else {
    if (a == MC_F2) launch_fspec_rows<MC_F2, MC_F2>(sc, ss, dc, ds, n, a, fail, g, st);
    else launch_fspec_rows<-1, MC_F2>(sc, ss, dc, ds, n, a, fail, g, st);
  }
}

}  // namespace

int mc_delta_decode_batch_impl(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                               size_t nchunks, size_t n, int astype, int dtype, int variant,
                               mc_stream_t stream);

extern "C" {

size_t mc_delta_decode_workspace(size_t n, int astype, int dtype) {
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

int mc_delta_decode(const void *src, void *dst, size_t n, int astype, int dtype, void *workspace,
                    size_t workspace_bytes, uint32_t *ticket, mc_stream_t stream) {
  if (ticket && (uintptr_t)ticket % 8) return MC_EINVAL;
  if (!mc_valid_dtype(dtype) || !mc_valid_dtype(astype)) return MC_EINVAL;
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
      launch_fspec_any(s, d, n, astype, dtype, workspace, st);
      return mc_last_launch();
    }
    launch_serial_any(s, 0, d, 0, n, 1, astype, dtype, st);
    return mc_last_launch();
  }
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  if (!workspace || workspace_bytes < mc_delta_decode_workspace(n, astype, dtype)) return MC_ENOSPC;
  uint64_t *sums = static_cast<uint64_t *>(workspace);
  if (astype == dtype && dtype != MC_B1 && ((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 16) == 0 &&
      dscan_enabled()) {
    const int es = mc_itemsize(dtype);
    // two launches with a ticket while groups stay <= 1024 tiles (the apply
    // workgroup sums its group's earlier tile totals, 4 per thread)
    if (ticket && es <= 4 && ds_group_tiles((n + (size_t)(32 / es) * MC_BLOCK - 1) / ((size_t)(32 / es) * MC_BLOCK)) <= 1024) {
      uint32_t *ws = static_cast<uint32_t *>(workspace);
      if (es == 1) launch_dscan_g<1>(s, d, n, ws, ticket, st);
      else if (es == 2) launch_dscan_g<2>(s, d, n, ws, ticket, st);
      else launch_dscan_g<4>(s, d, n, ws, ticket, st);
      return mc_last_launch();
    }
    switch (mc_itemsize(dtype)) {
      case 1: launch_dscan<1>(s, d, n, sums, st); break;
      case 2: launch_dscan<2>(s, d, n, sums, st); break;
      case 4: launch_dscan<4>(s, d, n, sums, st); break;
      default: launch_dscan<8>(s, d, n, sums, st); break;
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
      launch_serial_any(sc, src_stride, dc, dst_stride, n, rows, astype, dtype, st, variant);
      continue;
    }
    const size_t as = mc_itemsize(astype), ds = mc_itemsize(dtype);
    const bool vec = ((uintptr_t)sc % (4 * as) == 0) && (src_stride % (4 * as) == 0) &&
                     ((uintptr_t)dc % (4 * ds) == 0) && (dst_stride % (4 * ds) == 0);
    const bool al16 = ((uintptr_t)sc % 16 == 0) && (rows == 1 || src_stride % 16 == 0) &&
                      ((uintptr_t)dc % 16 == 0) && (rows == 1 || dst_stride % 16 == 0);
    if (astype == dtype && dtype != MC_B1 && al16 && dscan_enabled()) {
      const unsigned g = (unsigned)rows;
      switch (ds) {
        case 1: k_dscan_rows<1><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n); break;
        case 2: k_dscan_rows<2><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n); break;
        case 4: k_dscan_rows<4><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n); break;
        default: k_dscan_rows<8><<<g, MC_BLOCK, 0, st>>>(sc, src_stride, dc, dst_stride, n); break;
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
