// mc_scan.hip -- Delta decode = np.cumsum(enc, out=dec) (delta.py:69-83).
//
// numpy accumulates in the output dtype (add.accumulate with otype = dtype):
//   * integer dtypes: wrap-around addition, associative, so a parallel scan is
//     bit-exact.  Three passes over 4096-element tiles: per-tile totals, an
//     exclusive scan of the totals (one workgroup), then each tile rescanned
//     with its prefix (tile-local scans: lane-serial over 4 elements, wave
//     __shfl_up scan, LDS across the 4 waves).
//   * bool: numpy's bool add loop is logical or -- also associative.
//   * float dtypes: numpy adds left to right with a rounding after every add;
//     no reassociation reproduces that, so the float path keeps the serial
//     order exactly: one wave streams 1024-element blocks into LDS with
//     coalesced loads and lane 0 runs the dependent adds.  Bit-exact, not fast
//     (the integer-Delta pipeline is the bench path).
#include "mc_num.h"

namespace {

constexpr int TILE = 4096;  // elements per tile (256 threads x 4 steps x 4)
constexpr int STEPS = 4;

template <bool OR_OP>
MC_DEV uint64_t combine(uint64_t a, uint64_t b) {
  if constexpr (OR_OP) return a | b;
  else return a + b;
}

// value of element i as the accumulation type (dtype d, from astype a)
MC_DEV uint64_t scan_in(const uint8_t *src, size_t i, int a, int d, int as) {
  const McNum v = mc_num_cast(mc_num_from_bits(mc_load_elem_u(src, i, as), a), a, d);
  return (uint64_t)v.i;
}

template <bool OR_OP>
MC_DEV uint64_t wave_incl_scan(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t o = __shfl_up(v, off, 64);
    if (lane >= off) v = combine<OR_OP>(v, o);
  }
  return v;
}

// exclusive scan across the 256 threads of a block; returns the exclusive
// prefix for this thread, *total = block total
template <bool OR_OP>
MC_DEV uint64_t block_excl_scan(uint64_t v, uint64_t *lds, uint64_t *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan<OR_OP>(v);
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  uint64_t wpre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) {
    if (w < wave) wpre = combine<OR_OP>(wpre, lds[w]);
    tot = combine<OR_OP>(tot, lds[w]);
  }
  __syncthreads();
  *total = tot;
  // exclusive = inclusive minus own value (for OR: recompute exclusively)
  const uint64_t excl_in_wave = __shfl_up(incl, 1, 64);
  return combine<OR_OP>(wpre, lane ? excl_in_wave : 0);
}

template <bool OR_OP>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_reduce(const uint8_t *__restrict__ src,
                                                          size_t n, int a, int d,
                                                          uint64_t *__restrict__ sums) {
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const int as = mc_itemsize(a);
  const size_t base = (size_t)blockIdx.x * TILE;
  uint64_t acc = 0;
#pragma unroll
  for (int s = 0; s < STEPS; ++s)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t i = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x + k;
      if (i < n) acc = combine<OR_OP>(acc, scan_in(src, i, a, d, as));
    }
  uint64_t tot;
  block_excl_scan<OR_OP>(acc, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of ntiles tile totals in place (one workgroup of 1024)
template <bool OR_OP>
__global__ __launch_bounds__(1024) void k_scan_sums(uint64_t *sums, size_t ntiles) {
  __shared__ uint64_t lds[1024 / 64];
  const size_t per = (ntiles + 1023) / 1024;
  const size_t lo = threadIdx.x * per, hi = min(ntiles, lo + per);
  uint64_t acc = 0;
  for (size_t i = lo; i < hi; ++i) acc = combine<OR_OP>(acc, sums[i]);
  // block exclusive scan over 1024 threads (16 waves)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan<OR_OP>(acc);
  if (lane == 63) lds[wave] = incl;
  __syncthreads();
  uint64_t wpre = 0;
  for (int w = 0; w < wave; ++w) wpre = combine<OR_OP>(wpre, lds[w]);
  const uint64_t excl_in_wave = __shfl_up(incl, 1, 64);
  uint64_t run = combine<OR_OP>(wpre, lane ? excl_in_wave : 0);
  for (size_t i = lo; i < hi; ++i) {
    const uint64_t v = sums[i];
    sums[i] = run;
    run = combine<OR_OP>(run, v);
  }
}

template <bool OR_OP>
__global__ __launch_bounds__(MC_BLOCK) void k_scan_apply(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t n,
                                                         int a, int d,
                                                         const uint64_t *__restrict__ sums) {
  __shared__ uint64_t lds[MC_BLOCK / 64];
  const int as = mc_itemsize(a), ds = mc_itemsize(d);
  const size_t base = (size_t)blockIdx.x * TILE;
  uint64_t carry = sums[blockIdx.x];
#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
    const size_t i0 = base + (size_t)s * 4 * MC_BLOCK + 4 * (size_t)threadIdx.x;
    uint64_t p[4];
    uint64_t run = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < n) run = combine<OR_OP>(run, scan_in(src, i0 + k, a, d, as));
      p[k] = run;
    }
    uint64_t tot;
    const uint64_t excl = block_excl_scan<OR_OP>(run, lds, &tot);
    const uint64_t pre = combine<OR_OP>(carry, excl);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i0 + k < n)
        mc_store_elem_u(dst, i0 + k, ds, (uint64_t)mc_wrap((int64_t)combine<OR_OP>(pre, p[k]), d));
    carry = combine<OR_OP>(carry, tot);
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

}  // namespace

extern "C" {

size_t mc_delta_decode_workspace(size_t n, int astype, int dtype) {
  (void)astype;
  if (mc_is_float(dtype)) return 0;
  return ((n + TILE - 1) / TILE) * sizeof(uint64_t);
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
  const size_t ntiles = (n + TILE - 1) / TILE;
  if (!workspace || workspace_bytes < ntiles * sizeof(uint64_t)) return MC_ENOSPC;
  uint64_t *sums = static_cast<uint64_t *>(workspace);
  const bool or_op = dtype == MC_B1;
  if (or_op) {
    k_scan_reduce<true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, n, astype, dtype, sums);
    k_scan_sums<true><<<1, 1024, 0, st>>>(sums, ntiles);
    k_scan_apply<true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, astype, dtype, sums);
  } else {
    k_scan_reduce<false><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, n, astype, dtype, sums);
    k_scan_sums<false><<<1, 1024, 0, st>>>(sums, ntiles);
    k_scan_apply<false><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, n, astype, dtype, sums);
  }
  return mc_last_launch();
}

}  // extern "C"
