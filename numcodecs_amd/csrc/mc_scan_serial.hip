// mc_scan_serial.hip -- float Delta decode as numpy's serial chain (the
// path for inputs the speculative decode does not take, and for batches of
// chunks through mc_delta_decode_batch); its own translation unit so that
// it builds in parallel with mc_scan.hip.
#include "mc_scan.h"

namespace {

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
constexpr int SER_UN = 8;              // vectors of 4 elements in flight per lane

// L: numpy's loop dtype for cumsum(enc: A, out=dec: D) is
// np.promote_types(A, D) (mc_float_loop_dtype): the running sum is kept in L
// and each result is cast to D on output (f8 input into f4 output
// accumulates in f8; f2 output of f4 input accumulates in f4).  The fix-up
// mode (startp) reads its carry back from dst, so it needs L == D.
// SWO: the output dtype is big-endian (a big-endian input arrives as a
// flagged runtime astype, A_ = -1)
template <int A_, int D, bool VEC, int SER_SLOT_BYTES = 32768, int SER_G = 16, int L = D, bool SWO = false>
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
      uint64_t cb = mc_load_elem_u(dst, s0 - 1, DS);
      if constexpr (SWO) cb = mc_bswap_n(cb, DS);
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
        o[k] = j + k < cnt ? (L == D ? mc_num_to_bits(mc_num_f((double)p[j + k]), D | (SWO ? MC_BIG_ENDIAN : 0))
                                     : mc_num_to_bits(mc_num_cast(mc_num_f((double)p[j + k]), L, D),
                                                      D | (SWO ? MC_BIG_ENDIAN : 0)))
                           : 0;
      if (VEC && j + 4 <= cnt) {
        mc_store4(dst + (b0 + j) * DS, DS, o);
      } else {
        for (int k = 0; k < 4 && j + k < cnt; ++k) mc_store_elem_u(dst, b0 + j + k, DS, o[k]);
      }
    }
  };

  // same-type little-endian f4 / f8 with vector access: ser_chain_vbc for f4
  // when src and dst are equally 16-B aligned (as in k_fspec_walk's
  // fsw_stream); otherwise the LDS-fed chain below,
  // whose chain lane stores its results straight to dst (16-B global
  // stores) while the I/O wave only loads -- the chain's LDS writes were on
  // its critical path (13.1 -> 11.0 cycles per element, tools/probe_chain.py
  // kinds 1 and 14)
  constexpr bool DIRECT = L == D && A_ == D && VEC && !SWO && D != MC_F2;
  __shared__ size_t nan_at;  // first block whose chain ended NaN (ser_nan_fix)
  __shared__ unsigned long long nan_k0;
  if (threadIdx.x == 0) nan_at = SER_NO_NAN;
  if constexpr (DIRECT) {
    if (sizeof(T) == 4 && ((uintptr_t)src & 15) == ((uintptr_t)dst & 15)) {
      // one chain over the whole chunk by wave 0, straight from src to dst
      // (ser_chain_vbc); the I/O wave has nothing to stage
      if (!io) {
        const T *in = reinterpret_cast<const T *>(src);
        T *out = reinterpret_cast<T *>(dst);
        T acc = has_carry ? ser_add<L>(carry, in[0]) : in[0];
        out[0] = acc;
        acc = ser_chain_vbc<T, sizeof(T) == 8 ? 16 : 32, 6>(in + 1, out + 1, n - 1, acc);
        if (threadIdx.x == 0 && __builtin_isnan(acc)) nan_at = 0;
      }
      __syncthreads();
      if (nan_at != SER_NO_NAN) ser_nan_fix<L>(src, a, dst, D, n, 0, &nan_k0);
      return;
    }
  }
  if (io) load_blk(0);
  __syncthreads();
  T acc = 0;
  for (size_t b = 0; b < nb; ++b) {
    if (io) {
      if (!DIRECT && b >= 1) store_blk(b - 1);
      if (b + 1 < nb) load_blk(b + 1);
    } else if (lane == 0) {
      // software-pipelined chain: group g+1's LDS reads are in flight while
      // group g's adds run (ds_read latency ~50 cycles vs ~G dependent adds)
      T *p = slot[b & 1];
      T *o = DIRECT ? reinterpret_cast<T *>(dst + b * BLK * (size_t)DS) : p;
      const int cnt = (int)min((size_t)BLK, n - b * BLK);
      int j = 0;
      if (b == 0) {  // out[0] = x[0] exactly (no add), then align to a group
        acc = has_carry ? ser_add<L>(carry, p[0]) : p[0];
        o[0] = acc;
        const int m = cnt < SER_G ? cnt : SER_G;
        for (int k = 1; k < m; ++k) {
          acc = ser_add<L>(acc, p[k]);
          o[k] = acc;
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
          acc = ser_group<L, SER_G>(acc, ga);
          ser_st<T, SER_G>(o + j, ga);
          ser_ld<T, SER_G>(p + j + 2 * SER_G, ga);
          __builtin_amdgcn_sched_barrier(0);
          acc = ser_group<L, SER_G>(acc, gb);
          ser_st<T, SER_G>(o + j + SER_G, gb);
        }
      }
      for (; j < cnt; ++j) {
        acc = ser_add<L>(acc, p[j]);
        o[j] = acc;
      }
      if (L != MC_F2 && nan_at == SER_NO_NAN && __builtin_isnan(acc)) nan_at = b * BLK;
    }
    __syncthreads();
  }
  if (io && !DIRECT) store_blk(nb - 1);
  if constexpr (L != MC_F2) {  // numpy's NaN tail (f2 chains are exact in-chain)
    __syncthreads();
    if (nan_at != SER_NO_NAN) ser_nan_fix<L>(src, a, dst, D | (SWO ? MC_BIG_ENDIAN : 0), n, nan_at, &nan_k0);
  }
}

// (slot bytes, group) per schedule: a 32 KiB slot amortises the block
// barrier for one long chain; a batch needs small slots so that many chains
// (workgroups) fit a CU's LDS at once (2 x 32 KiB slots allow only 2).

// big-endian output (swo): the generic-input instantiations with SWO; a
// big-endian input arrives flagged in `a` and takes the A_ = -1 paths
template <int D, int L>
static void launch_serial_be(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n, size_t rows, int a,
                             bool v, hipStream_t st) {
  const unsigned g = (unsigned)rows;
  const int slot = rows >= 256 ? 8192 : 32768;
  if (v && slot == 8192) k_scan_serial<-1, D, true, 8192, 16, L, true><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
  else if (v) k_scan_serial<-1, D, true, 32768, 32, L, true><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
  else k_scan_serial<-1, D, false, 8192, 16, L, true><<<g, 128, 0, st>>>(s, ss, d, dss, n, a);
}

template <int D>
static void launch_serial(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n,
                          size_t rows, int a, hipStream_t st, int variant = 0, bool swo = false) {
  const int as = mc_itemsize(a);
  const int loop = mc_float_loop_dtype(a, D);
  if (swo) {
    const bool v = ((uintptr_t)s % (4 * as) == 0) && (ss % (4 * as) == 0) &&
                   ((uintptr_t)d % (4 * mc_itemsize(D)) == 0) && (dss % (4 * mc_itemsize(D)) == 0);
    if (loop == D) launch_serial_be<D, D>(s, ss, d, dss, n, rows, a, v, st);
    else if constexpr (D != MC_F8) {
      if (loop == MC_F8) launch_serial_be<D, MC_F8>(s, ss, d, dss, n, rows, a, v, st);
      else if constexpr (D == MC_F2) launch_serial_be<D, MC_F4>(s, ss, d, dss, n, rows, a, v, st);
    }
    return;
  }
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

}  // namespace

void mc_launch_serial_any(const uint8_t *s, size_t ss, uint8_t *d, size_t dss, size_t n, size_t rows, int a, int dt,
                          hipStream_t st, int variant) {
  const bool swo = mc_dt_swapped(dt);
  dt = mc_dt_base(dt);
  if (dt == MC_F8) launch_serial<MC_F8>(s, ss, d, dss, n, rows, a, st, variant, swo);
  else if (dt == MC_F4) launch_serial<MC_F4>(s, ss, d, dss, n, rows, a, st, variant, swo);
  else launch_serial<MC_F2>(s, ss, d, dss, n, rows, a, st, variant, swo);
}
