// lab_dscan_reduce.hip -- LAB ONLY (libmcodec_lab.so): the same-width integer
// Delta decode's reduce pass (k_dscan_reduce_g, ES = 2, whole tiles only)
// restated two ways for tools/probe_dscan_reduce.py:
//   PERSIST = false: one workgroup per group of 4 tiles (the product's shape,
//                    8192 short-lived workgroups for 256 MiB);
//   PERSIST = true:  a capped grid of workgroups looping over the groups,
//                    the next group's loads issued before this group's sums
//                    and arrival atomic (the shape of the round-6 verifies).
// Both write the same tile totals, group totals and leave the ticket zero.
#include "mc_common.h"

namespace {

typedef unsigned short lab_ushort2 __attribute__((ext_vector_type(2)));
constexpr int LG = 4;           // tiles per group (DS_GROUP)
constexpr size_t LTB = 8192;    // tile bytes: 16 int16 per lane x 256 lanes

template <bool PERSIST>
__global__ __launch_bounds__(MC_BLOCK) void k_lab_dsr(const uint8_t *__restrict__ src, size_t ngroups,
                                                      uint32_t *__restrict__ ws, uint32_t *ticket, size_t ntiles,
                                                      unsigned GT) {
  __shared__ uint32_t lds[2][LG][MC_BLOCK / 64];
  uint32_t *tile_tot = ws, *gtot = ws + ntiles;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto load = [&](mc_u32x4 (&v)[2 * LG], size_t grp) {
#pragma unroll
    for (int h = 0; h < LG; ++h) {
      const uint8_t *tb = src + (grp * LG + h) * LTB;
      v[2 * h] = mc_ld16<false>(tb + 16 * (size_t)threadIdx.x);
      v[2 * h + 1] = mc_ld16<false>(tb + 16 * (size_t)(MC_BLOCK + threadIdx.x));
    }
  };
  auto fold = [&](const mc_u32x4 (&v)[2 * LG], size_t grp, int par) {
    uint32_t acc[LG];
#pragma unroll
    for (int h = 0; h < LG; ++h) {
      const uint32_t d[8] = {v[2 * h].x, v[2 * h].y, v[2 * h].z, v[2 * h].w,
                             v[2 * h + 1].x, v[2 * h + 1].y, v[2 * h + 1].z, v[2 * h + 1].w};
      uint32_t a = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) a = __builtin_amdgcn_udot2(__builtin_bit_cast(lab_ushort2, d[i]), lab_ushort2{1, 1}, a, false);
      acc[h] = a;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int h = 0; h < LG; ++h) acc[h] += __shfl_xor(acc[h], off, 64);
    if (lane == 0) {
#pragma unroll
      for (int h = 0; h < LG; ++h) lds[par][h][wave] = acc[h];
    }
    __syncthreads();  // lds[par] is rewritten two groups later, after the next barrier
    if (threadIdx.x != 0) return;
    const size_t t0 = grp * LG;
    uint32_t tot = 0;
    for (int h = 0; h < LG; ++h) {
      uint32_t a = 0;
      for (int w = 0; w < MC_BLOCK / 64; ++w) a += lds[par][h][w];
      tile_tot[t0 + h] = a;
      tot += a;
    }
    const size_t g = t0 / GT;
    const size_t in_group = ntiles - g * GT < GT ? ntiles - g * GT : GT;
    const unsigned long long arrivals = (in_group + LG - 1) / LG;
    unsigned long long *word = reinterpret_cast<unsigned long long *>(ticket + (size_t)MC_ARRIVAL_LINE * g);
    const unsigned long long old = atomicAdd(word, ((unsigned long long)tot << 16) | 1ull);
    if ((old & 0xffffu) + 1u == arrivals) {
      gtot[g] = (uint32_t)(old >> 16) + tot;
      *word = 0;
    }
  };
  mc_u32x4 a[2 * LG], b[2 * LG];
  size_t grp = blockIdx.x;
  if constexpr (!PERSIST) {
    load(a, grp);
    fold(a, grp, 0);
    return;
  }
  if (grp < ngroups) load(a, grp);
  while (grp < ngroups) {
    const size_t g1 = grp + gridDim.x;
    if (g1 < ngroups) load(b, g1);
    fold(a, grp, 0);
    if (g1 >= ngroups) break;
    const size_t g2 = g1 + gridDim.x;
    if (g2 < ngroups) load(a, g2);
    fold(b, g1, 1);
    grp = g2;
  }
}

}  // namespace

// nbytes: a multiple of 32 KiB (whole groups of int16 tiles); ws: ntiles + 64
// words; ticket: MC_ARRIVAL_WORDS zero words (left zero)
extern "C" int mc_lab_dscan_reduce(const void *src, size_t nbytes, uint32_t *ws, uint32_t *ticket, int persist,
                                   unsigned grid, mc_stream_t stream) {
  if (!src || !ws || !ticket || nbytes == 0 || nbytes % (LG * LTB) || ((uintptr_t)src & 15)) return MC_EINVAL;
  const size_t ntiles = nbytes / LTB, ngroups = ntiles / LG;
  unsigned gt = 256;
  while ((ntiles + gt - 1) / gt > 64) gt *= 2;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  hipStream_t st = (hipStream_t)stream;
  if (persist) {
    const unsigned g = (unsigned)(grid == 0 || grid > ngroups ? ngroups : grid);
    k_lab_dsr<true><<<g, MC_BLOCK, 0, st>>>(s, ngroups, ws, ticket, ntiles, gt);
  } else {
    k_lab_dsr<false><<<(unsigned)ngroups, MC_BLOCK, 0, st>>>(s, ngroups, ws, ticket, ntiles, gt);
  }
  return mc_last_launch();
}
