// lab_ck_stamp.hip -- LAB ONLY (libmcodec_lab.so): the one-launch CRC verify
// (mcck::k_crc_tiles_bs FUSED, checksum only, 16-B aligned source) restated
// with wall_clock64() stamps (100 MHz), to locate the 10-12 us between the
// checksum-only tile pass (41.5 us) and the one-launch verify (52-54 us):
//   per workgroup (4 words): start, tile loop done, partial stores drained
//   (vmcnt), arrival atomic returned;
//   the last arriver (8 words after the grid's): LDS tables built, partial
//   loads back, fold + lane reduce done, thread 0's finish done, verdict
//   published.
// tools/probe_ck_stamp.py times it against the product entry point and
// prints the breakdown.
#include "mc_checksum.h"

namespace mcck {
namespace {

template <int KIND, int K>
__global__ __launch_bounds__(MC_BLOCK, 2) void k_lab_crc_stamp(const uint8_t *__restrict__ src, size_t n,
                                                               size_t total, uint32_t *__restrict__ partials,
                                                               const CrcFin fin, const CkFinish fx,
                                                               unsigned long long *__restrict__ stamps) {
  __shared__ uint32_t red[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long *my = stamps + 4 * (size_t)blockIdx.x;
  if (threadIdx.x == 0) my[0] = wall_clock64();
  uint32_t gx[32];
  gx[0] = crc_consts<KIND>().g[threadIdx.x];
#pragma unroll
  for (int i = 1; i < 32; ++i) gx[i] = mulx_r<KIND>(gx[i - 1]);
  constexpr size_t TB = (size_t)K * STEP;
  auto load = [&](mc_u32x4 (&v)[K], size_t tile) {
    ck_load_tile<K, 2>(v, src, tile * TB + 16 * (size_t)threadIdx.x, n, (tile + 1) * TB <= n);
  };
  auto fold = [&](const mc_u32x4 (&v)[K], size_t tile, int par) {
    const uint32_t acc = crc_fold_bs<KIND, K>(v);
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i)
      p = __builtin_amdgcn_bitop3_b32(p, (uint32_t)__builtin_amdgcn_sbfe((int)acc, 31 - i, 1), gx[i], 0x78);
    p = wave_xor(p);
    if (lane == 0) red[par][wave] = p;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0;
#pragma unroll
      for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= red[par][w];
      __hip_atomic_store(&partials[tile], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  mc_u32x4 a[K], b[K];
  size_t tile = blockIdx.x;
  if (tile < total) load(a, tile);
  while (tile < total) {
    const size_t t1 = tile + gridDim.x;
    if (t1 < total) load(b, t1);
    fold(a, tile, 0);
    if (t1 >= total) break;
    const size_t t2 = t1 + gridDim.x;
    if (t2 < total) load(a, t2);
    fold(b, t1, 1);
    tile = t2;
  }
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {
    my[1] = wall_clock64();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    my[2] = wall_clock64();
    last = mc_arrive_last(fx.ticket, gridDim.x);
    my[3] = wall_clock64();
  }
  __syncthreads();
  if (!last) return;
  unsigned long long *ls = stamps + 4 * (size_t)gridDim.x;
  // ck_finish_chunk<KIND, K, true> (CRC branch) with stamps
  __shared__ uint32_t T[4][256];
  __shared__ uint32_t lred[MC_BLOCK / 64];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if ((threadIdx.x >> k) & 1) r ^= fin.xb[8 * j + k];
    T[j][threadIdx.x] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) ls[0] = wall_clock64();
  const size_t lo = total * threadIdx.x / MC_BLOCK, hi = total * (threadIdx.x + 1) / MC_BLOCK;
  constexpr int B = 16;
  uint32_t acc = 0;
  bool stamped = false;
  for (size_t j0 = lo; j0 < hi; j0 += B) {
    uint32_t v[B];
#pragma unroll
    for (int u = 0; u < B; ++u) v[u] = ck_ld<true>(&partials[j0 + u < hi ? j0 + u : hi - 1]);
    if (threadIdx.x == 0 && !stamped) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ls[1] = wall_clock64();
      stamped = true;
    }
#pragma unroll
    for (int u = 0; u < B; ++u)
      if (j0 + u < hi)
        acc = (T[0][acc & 0xffu] ^ T[1][(acc >> 8) & 0xffu] ^ T[2][(acc >> 16) & 0xffu] ^ T[3][acc >> 24]) ^ v[u];
  }
  if (hi > lo) acc = gf_mul(acc, fin.tail[threadIdx.x], crc_poly<KIND>());
  acc = wave_xor(acc);
  if (lane == 0) lred[wave] = acc;
  __syncthreads();
  if (threadIdx.x != 0) return;
  ls[2] = wall_clock64();
  uint32_t r = 0;
  for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= lred[w];
  r = gf_mul(r, fin.pad, crc_poly<KIND>());
  if (fin.head) {
    uint32_t hw = load_le32(fx.stored);
#pragma unroll
    for (int i = 0; i < 32; ++i) hw = (hw >> 1) ^ ((hw & 1u) ? crc_poly<KIND>() : 0u);
    r ^= gf_mul(hw, fin.xn, crc_poly<KIND>());
  }
  const uint32_t result = ~(gf_mul(~fx.init, fin.xn, crc_poly<KIND>()) ^ r);
  ls[3] = wall_clock64();
  if (fx.stored_out) fx.stored_out[0] = load_le32(fx.stored);
  if (fx.out) fx.out[0] = result;
  mc_publish_verdict_seq(fx.out, fx.seq);
  ls[4] = wall_clock64();
  mc_arrivals_reset(fx.ticket);
}

}  // namespace

// host: the product's CrcFin for (K = 16, tpc, n, np) -- restated here from
// crc_fin_build (mc_checksum.hip keeps it in an anonymous namespace)
template <int KIND>
CrcFin lab_fin(int K, size_t tpc, size_t n, size_t np) {
  CrcFin f{};
  f.head = n != np;
  constexpr uint32_t poly = crc_poly<KIND>();
  auto pw = [&](uint32_t base, uint64_t e) {
    uint32_t p = GF_ONE, b = base;
    for (; e; e >>= 1) {
      if (e & 1) p = gf_mul(p, b, poly);
      b = gf_mul(b, b, poly);
    }
    return p;
  };
  const uint32_t xinv = (poly << 1) | 1u;
  const uint32_t X = pw(GF_X, 8 * (uint64_t)K * STEP);
  for (int m = 0; m < 32; ++m) f.xb[m] = gf_mul(1u << m, X, poly);
  for (int t = 0; t < MC_BLOCK; ++t) f.tail[t] = pw(X, tpc - tpc * (t + 1) / MC_BLOCK);
  f.pad = pw(xinv, 8 * ((uint64_t)K * STEP * tpc - n));
  f.xn = pw(GF_X, 8 * (uint64_t)np);
  return f;
}

}  // namespace mcck

// one-launch CRC verify of `encoded_bytes` at a 16-B aligned `src` with the
// stored word at the start (location "start"): out_pair {computed, stored};
// stamps: 4 * grid + 8 words
extern "C" int mc_lab_crc_verify_stamp(int kind, const void *src, size_t encoded_bytes, uint32_t init,
                                       uint32_t *out_pair, uint32_t seq, void *ws, uint32_t *ticket, unsigned grid,
                                       unsigned long long *stamps, mc_stream_t stream) {
  using namespace mcck;
  if (!src || ((uintptr_t)src & 15) || encoded_bytes < 65536 || !ws || !ticket || !stamps || grid == 0)
    return MC_EINVAL;
  const size_t n = encoded_bytes, np = encoded_bytes - 4;
  constexpr int K = 16;
  const size_t total = (n + (size_t)K * STEP - 1) / ((size_t)K * STEP);
  if (grid > total) grid = (unsigned)total;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  const CkFinish fx{init, seq, 4, ticket, out_pair, out_pair + 1, nullptr, 0, s};
  hipStream_t st = (hipStream_t)stream;
  uint32_t *parts = static_cast<uint32_t *>(ws);
  if (kind == MC_CK_CRC32)
    k_lab_crc_stamp<K_CRC32, K><<<grid, MC_BLOCK, 0, st>>>(s, n, total, parts, lab_fin<K_CRC32>(K, total, n, np),
                                                           fx, stamps);
  else if (kind == MC_CK_CRC32C)
    k_lab_crc_stamp<K_CRC32C, K><<<grid, MC_BLOCK, 0, st>>>(s, n, total, parts, lab_fin<K_CRC32C>(K, total, n, np),
                                                            fx, stamps);
  else
    return MC_EINVAL;
  return mc_last_launch();
}
