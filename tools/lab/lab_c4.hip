// lab_c4.hip -- LAB ONLY (libmcodec_lab.so, built by tools/lab/Makefile from
// the product objects plus this file; never part of libmcodec.so or
// include/mcodec.h).  Alternative decode schedules of the fused
// FSO -> Delta -> Shuffle(2) chunk pipeline that DESIGN.md measured against
// the product's 3-pass scan and rejected, kept so the measurement can be
// repeated and so their byte-identity stays tested (tests/test_gpu_c4.py):
//   1  the product's three-pass scan (= 0; the product's default is the
//      two-launch decode, mc_fso_delta_shuffle_decode with a ticket)
//   2  single-pass decoupled look-back, tiles numbered by an atomic counter
//   3  single-pass look-back in workgroup (blockIdx) order
//   4  = 3 with every wait replaced by the data-derived prefix fallback
//   5/6 single-pass look-back over partitions of 4 / 8 tiles in registers
//   7  = 5 with the forced fallback
// Variant 3 and 5/6 rely on workgroups being dispatched roughly in blockIdx
// order for SPEED only: a predecessor that stays unpublished past the spin
// bound makes the tile derive its prefix from the data itself.
#include "lab_lookback.h"
#include "mc_c4.h"

namespace {

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

}  // namespace


extern "C" {

size_t mc_lab_c4_decode_workspace(size_t n) {
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const size_t prod = mc_fso_delta_shuffle_decode_workspace(n);
  return mc_lb_workspace(ntiles) > prod ? mc_lb_workspace(ntiles) : prod;
}

// variant 0 / 1: the product's three-pass scan; 2-7 as listed above (the
// partition-in-LDS single pass is mc_lab_c4_dec1p, lab_scan1p.hip).
// Identical bytes.
int mc_lab_c4_decode_variant(const void *src, void *dst, size_t n, int astype, int dtype, double scale,
                             double offset, void *workspace, size_t workspace_bytes, int variant,
                             mc_stream_t stream) {
  if (variant < 0 || variant > 7) return MC_EINVAL;
  if (variant <= 1)
    return mc_fso_delta_shuffle_decode(src, dst, n, astype, dtype, scale, offset, workspace, workspace_bytes,
                                       nullptr, stream);
  if (n == 0) return MC_OK;
  if (!c4_ok(src, dst, n, dtype, astype)) return MC_EINVAL;
  if (!workspace || workspace_bytes < mc_lab_c4_decode_workspace(n)) return MC_ENOSPC;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  hipStream_t st = (hipStream_t)stream;
  uint8_t *ws = static_cast<uint8_t *>(workspace);
  const size_t ntiles = (n + MC_SCAN_TILE - 1) / MC_SCAN_TILE;
  const int rc = mc_hip_status(hipMemsetAsync(ws, 0, mc_lb_workspace(ntiles), st));
  if (rc != MC_OK) return rc;
  if (variant >= 5) {
    const unsigned spins = variant == 7 ? 0u : MC_LB_WAVE_SPINS;
    const int R = variant == 6 ? 8 : 4;
    MC_C4_DISPATCH(c4_decode_lbp, s, d, ws, p, R, spins, st);
  } else {
    // variant 4: no waiting at all, every tile whose predecessor has not
    // published yet takes the data-derived fallback
    const unsigned spins = variant == 4 ? 0u : MC_LB_WAVE_SPINS;
    MC_C4_DISPATCH(c4_decode_lb, s, d, ws, p, variant == 2, spins, st);
  }
  return mc_last_launch();
}

}  // extern "C"
