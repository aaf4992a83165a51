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
//     order exactly: one wave streams 1024-element blocks into LDS with
//     coalesced loads and lane 0 runs the dependent adds.  Bit-exact, not fast
//     (the integer-Delta pipeline is the bench path).
#include "mc_scan.h"

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

// float dtypes: exact left-to-right accumulation (one wave)
constexpr int SER_BLK = 1024;

__global__ __launch_bounds__(64) void k_scan_serial(const uint8_t *__restrict__ src,
                                                    uint8_t *__restrict__ dst, size_t n, int a,
                                                    int d) {
  __shared__ uint64_t buf[SER_BLK];
  const int as = mc_itemsize(a), ds = mc_itemsize(d);
  const int lane = threadIdx.x;
  McNum acc = mc_num_f(0.0);
  for (size_t b0 = 0; b0 < n; b0 += SER_BLK) {
    const size_t cnt = min((size_t)SER_BLK, n - b0);
    for (int j = lane; j < (int)cnt; j += 64) buf[j] = mc_load_elem_u(src, b0 + j, as);
    __syncthreads();
    if (lane == 0) {
      for (int j = 0; j < (int)cnt; ++j) {
        const McNum x = mc_num_cast(mc_num_from_bits(buf[j], a), a, d);
        acc = (b0 + j == 0) ? x : mc_num_binop(acc, x, MC_OP_ADD, d);
        buf[j] = mc_num_to_bits(acc, d);
      }
    }
    __syncthreads();
    for (int j = lane; j < (int)cnt; j += 64) mc_store_elem_u(dst, b0 + j, ds, buf[j]);
    __syncthreads();
  }
}

template <bool OR_OP, int A_, int D_, bool VEC>
static void launch_int_scan(const uint8_t *s, uint8_t *d, size_t n, int a, int dt, uint64_t *sums,
                            size_t ntiles, hipStream_t st) {
  k_scan_reduce<OR_OP, A_, D_, VEC><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, n, a, dt, sums);
  mc_launch_scan_sums<OR_OP>(sums, ntiles, st);
  k_scan_apply<OR_OP, A_, D_, VEC><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, a, dt, sums);
}

}  // namespace

extern "C" {

size_t mc_delta_decode_workspace(size_t n, int astype, int dtype) {
  (void)astype;
  if (mc_is_float(dtype)) return 0;
  return ((n + MC_SCAN_TILE - 1) / MC_SCAN_TILE) * sizeof(uint64_t);
}

int mc_delta_decode(const void *src, void *dst, size_t n, int astype, int dtype, void *workspace,
                    size_t workspace_bytes, mc_stream_t stream) {
  if (!mc_valid_dtype(dtype) || !mc_valid_dtype(astype)) return MC_EINVAL;
  if (n == 0) return MC_OK;
  if (!src || !dst) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  if (mc_is_float(dtype)) {
    k_scan_serial<<<1, 64, 0, st>>>(s, d, n, astype, dtype);
    return mc_last_launch();
  }
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  if (!workspace || workspace_bytes < ntiles * sizeof(uint64_t)) return MC_ENOSPC;
  uint64_t *sums = static_cast<uint64_t *>(workspace);
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

}  // extern "C"
