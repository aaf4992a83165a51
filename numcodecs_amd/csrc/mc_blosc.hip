// mc_blosc.hip -- Blosc's shuffle filters applied block by block (SURVEY.md
// §8f row 2; blosc.pyx:67-71 NOSHUFFLE/SHUFFLE/BITSHUFFLE, :211-326), with
// c-blosc 1.x semantics pinned by the reference's fixture/blosc frames
// (oracle/blosc.py):
//   * the buffer is cut into `blocksize`-byte blocks (the last one shorter),
//     each filtered on its own, E = bsize / typesize elements per block;
//   * SHUFFLE: byte transpose of the (E, typesize) matrix, the bsize %
//     typesize trailing bytes copied -- run on the Shuffle kernels
//     (mc_shuffle.hip) as a batch of equal blocks plus the last block;
//   * BITSHUFFLE (bitshuffle's bshuf_trans_bit_elem): if E % 8 == 0, bit k of
//     byte j of element i -> bit i%8 of byte i/8 of bit-plane 8j+k (planes of
//     E/8 bytes); otherwise the block is copied unchanged.
//
// Bit-shuffle kernel: a workgroup owns G groups of 8 elements of one block
// (G*8*typesize <= 32 KiB).  The elements are staged in LDS with coalesced
// loads; thread t gathers, for every byte position j, byte j of its 8
// elements into a u64 and transposes that 8x8 bit matrix with three
// delta-swaps, giving the 8 plane bytes (8j+k, t); these are staged in LDS
// plane-major and leave as coalesced per-plane runs of G bytes.  The inverse
// runs the same steps backwards (the 8x8 transpose is an involution).
#include "mc_common.h"

namespace {

MC_DEV uint64_t tr8x8(uint64_t x) {  // byte r bit c  <->  byte c bit r
  uint64_t t;
  t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x = x ^ t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x = x ^ t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  x = x ^ t ^ (t << 28);
  return x;
}

constexpr int BS_LDS = 32768;  // bytes of element data per workgroup

inline unsigned groups_per_wg(size_t ts) {
  const size_t g = BS_LDS / (8 * ts);
  return (unsigned)(g < MC_BLOCK ? g : MC_BLOCK);
}

// copy [lo, hi) of a block, spread over the workgroup
MC_DEV void wg_copy(const uint8_t *s, uint8_t *d, size_t lo, size_t hi) {
  for (size_t i = lo + threadIdx.x; i < hi; i += MC_BLOCK) d[i] = s[i];
}

template <bool FWD>
__global__ __launch_bounds__(MC_BLOCK) void k_bitshuffle(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t nbytes,
                                                         unsigned ts, size_t blocksize,
                                                         unsigned G) {
  __shared__ __attribute__((aligned(16))) uint8_t elem[BS_LDS];
  __shared__ __attribute__((aligned(16))) uint8_t plane[BS_LDS];
  const size_t b0 = (size_t)blockIdx.x * blocksize;
  const size_t bsize = nbytes - b0 < blocksize ? nbytes - b0 : blocksize;
  const uint8_t *s = src + b0;
  uint8_t *d = dst + b0;
  const size_t E = bsize / ts;
  const size_t wg_bytes = (size_t)G * 8 * ts;
  const size_t lo = (size_t)blockIdx.y * wg_bytes;
  if (E % 8) {  // c-blosc copies such blocks unchanged
    if (lo < bsize) wg_copy(s, d, lo, lo + wg_bytes < bsize ? lo + wg_bytes : bsize);
    return;
  }
  if (blockIdx.y == 0) wg_copy(s, d, E * ts, bsize);  // trailing bytes, if any
  const size_t ng = E / 8, g0 = (size_t)blockIdx.y * G;
  if (g0 >= ng) return;
  const unsigned Gt = (unsigned)(ng - g0 < G ? ng - g0 : G);
  const unsigned n8 = 8 * ts;  // planes
  const size_t pstride = E / 8;
  const int t = threadIdx.x;
  if (FWD) {
    const size_t off = g0 * n8, len = (size_t)Gt * n8;
    if ((((uintptr_t)(s + off)) & 15) == 0 && (len & 15) == 0) {
      for (size_t i = 16 * (size_t)t; i < len; i += 16 * MC_BLOCK)
        *reinterpret_cast<mc_u32x4 *>(elem + i) = mc_ld16<true>(s + off + i);
    } else {
      for (size_t i = t; i < len; i += MC_BLOCK) elem[i] = s[off + i];
    }
    __syncthreads();
    if (t < (int)Gt) {
      for (unsigned j = 0; j < ts; ++j) {
        uint64_t x = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) x |= (uint64_t)elem[(8 * t + r) * ts + j] << (8 * r);
        x = tr8x8(x);
#pragma unroll
        for (int k = 0; k < 8; ++k) plane[(8 * j + k) * Gt + t] = (uint8_t)(x >> (8 * k));
      }
    }
    __syncthreads();
    for (unsigned i = t; i < n8 * Gt; i += MC_BLOCK) {
      const unsigned p = i / Gt, q = i - p * Gt;
      d[p * pstride + g0 + q] = plane[i];
    }
  } else {
    for (unsigned i = t; i < n8 * Gt; i += MC_BLOCK) {
      const unsigned p = i / Gt, q = i - p * Gt;
      plane[i] = s[p * pstride + g0 + q];
    }
    __syncthreads();
    if (t < (int)Gt) {
      for (unsigned j = 0; j < ts; ++j) {
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) x |= (uint64_t)plane[(8 * j + k) * Gt + t] << (8 * k);
        x = tr8x8(x);
#pragma unroll
        for (int r = 0; r < 8; ++r) elem[(8 * t + r) * ts + j] = (uint8_t)(x >> (8 * r));
      }
    }
    __syncthreads();
    const size_t off = g0 * n8, len = (size_t)Gt * n8;
    if ((((uintptr_t)(d + off)) & 15) == 0 && (len & 15) == 0) {
      for (size_t i = 16 * (size_t)t; i < len; i += 16 * MC_BLOCK)
        mc_st16<true>(d + off + i, *reinterpret_cast<const mc_u32x4 *>(elem + i));
    } else {
      for (size_t i = t; i < len; i += MC_BLOCK) d[off + i] = elem[i];
    }
  }
}


// ---------------------------------------------------------------------------
// Fast path for typesize ES in {1, 2, 4, 8} and blocks whose element count is
// a multiple of 32 (every plane then starts dword aligned): thread t owns 4
// consecutive groups of 8 elements (32*ES contiguous bytes) and writes one
// dword (4 groups) of each of its 8*ES planes -- 256 contiguous bytes per
// plane per wave store.  The element side moves through LDS with coalesced
// 16-B global accesses; the LDS image is XOR-swizzled per owner thread
// (slot i of thread t at 2ES*t + (i ^ (t & (2ES-1)))) so that the owner's
// ds_read/write_b128 sweep is at most 2-way bank conflicted.  Byte j of
// element e sits at bit 8*((e*ES + j) % 4) of dword (e*ES + j)/4 -- all
// compile-time, so the gathers become v_bfe/v_perm.
// ---------------------------------------------------------------------------
constexpr int BF_GPT = 4;                     // groups per thread
constexpr int BF_GROUPS = BF_GPT * MC_BLOCK;  // groups per workgroup

template <int ES>
MC_DEV int bf_slot(int t, int i) {
  return 2 * ES * t + (i ^ (t & (2 * ES - 1)));
}

template <int ES>
MC_DEV uint32_t bf_byte(const uint32_t (&w)[8 * ES], int e, int j) {
  const int b = e * ES + j;
  return (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
}

// 32 x 32 bit transpose, LSB first: afterwards bit c of a[r] is bit r of the
// input a[c].  With 32 consecutive elements of 4 bytes, row i = element i
// and output row p = bit-plane p's 4 bytes for those elements -- Blosc's
// bit-shuffle of the thread's 4 groups in one transpose (8-B elements: one
// per dword half).  The 16- and 8-bit stages are byte moves (v_perm_b32, 2
// per row pair), the 4/2/1-bit stages delta swaps (5 ops per pair): 304 VALU
// ops per 128 B, against ~1100 for the per-group gather / 8x8 transpose /
// scatter it replaces for ES = 4 and 8 (the kernel was issue-bound).
MC_DEV void tr32x32(uint32_t (&a)[32]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t x = a[k], y = a[k + 16];
    a[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);
    a[k + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);
  }
#pragma unroll
  for (int blk = 0; blk < 32; blk += 16)
#pragma unroll
    for (int k = blk; k < blk + 8; ++k) {
      const uint32_t x = a[k], y = a[k + 8];
      a[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);
      a[k + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);
    }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & 4) continue;
    const uint32_t t = __builtin_amdgcn_bitop3_b32(a[k] >> 4, a[k + 4], 0x0F0F0F0Fu, 0x28);  // (x ^ y) & m
    a[k + 4] ^= t;
    a[k] ^= t << 4;
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & 2) continue;
    const uint32_t t = __builtin_amdgcn_bitop3_b32(a[k] >> 2, a[k + 2], 0x33333333u, 0x28);
    a[k + 2] ^= t;
    a[k] ^= t << 2;
  }
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    const uint32_t t = __builtin_amdgcn_bitop3_b32(a[k] >> 1, a[k + 1], 0x55555555u, 0x28);
    a[k + 1] ^= t;
    a[k] ^= t << 1;
  }
}

// the thread's 8*ES plane dwords from its 32 elements' 8*ES dwords (ES = 4:
// one transpose; ES = 8: the low and the high dword of every element),
// stored as each half is ready (no second 8*ES-dword array: ES = 8 spilled)
template <int ES>
MC_DEV void bf_planes_store(const uint32_t (&w)[8 * ES], uint8_t *pd, size_t pstride) {
  static_assert(ES == 4 || ES == 8, "32x32 transposes for 4- and 8-byte elements");
#pragma unroll
  for (int h = 0; h < ES / 4; ++h) {
    uint32_t a[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = w[(ES / 4) * i + h];
    tr32x32(a);
#pragma unroll
    for (int p = 0; p < 32; ++p)
      __builtin_nontemporal_store(a[p], reinterpret_cast<uint32_t *>(pd + (size_t)(32 * h + p) * pstride));
  }
}

// ES = 1 / 2: per group of 8 elements, byte j of the 8 elements -> u64 ->
// 8x8 bit transpose -> byte k is plane 8j+k's byte for that group; the
// thread's 4 groups give one dword of each of its 8*ES planes
template <int ES>
MC_DEV void bf_planes_store_small(const uint32_t (&w)[8 * ES], uint8_t *pd, size_t pstride) {
#pragma unroll
  for (int j = 0; j < ES; ++j) {
    uint64_t T[BF_GPT];
#pragma unroll
    for (int g = 0; g < BF_GPT; ++g) {
      uint64_t x = 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) x |= (uint64_t)bf_byte<ES>(w, 8 * g + r, j) << (8 * r);
      T[g] = tr8x8(x);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t o = 0;
#pragma unroll
      for (int g = 0; g < BF_GPT; ++g) o |= (uint32_t)((T[g] >> (8 * k)) & 0xffu) << (8 * g);
      __builtin_nontemporal_store(o, reinterpret_cast<uint32_t *>(pd + (size_t)(8 * j + k) * pstride));
    }
  }
}
// and back: the thread's 8*ES plane dwords -> its 32 elements' 8*ES dwords
template <int ES>
MC_DEV void bf_elems_small(const uint32_t (&pl)[8 * ES], uint32_t (&w)[8 * ES]) {
#pragma unroll
  for (int i = 0; i < 8 * ES; ++i) w[i] = 0;
#pragma unroll
  for (int j = 0; j < ES; ++j) {
#pragma unroll
    for (int g = 0; g < BF_GPT; ++g) {
      uint64_t x = 0;  // byte k = plane 8j+k's byte for group g
#pragma unroll
      for (int k = 0; k < 8; ++k) x |= (uint64_t)((pl[8 * j + k] >> (8 * g)) & 0xffu) << (8 * k);
      x = tr8x8(x);  // byte r = byte j of element 8g+r
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int b = (8 * g + r) * ES + j;
        w[b >> 2] |= (uint32_t)((x >> (8 * r)) & 0xffu) << (8 * (b & 3));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pipelined bit-shuffle, every fast typesize (round 5).  The round-4 kernel ran one
// 32 KiB (64 KiB) tile per workgroup in three serial phases -- load, barrier,
// transpose + store -- and its waves spent 77 % of their cycles parked on the
// loads (SQ_WAIT_ANY, profiles/r05/bsh_pmc.txt) at ~13 resident waves per CU.
// Here a persistent grid of workgroups walks the tiles, and each thread's
// share of tile i + 1 is loaded into registers while tile i is transposed and
// stored, so the loads' latency hides behind the previous tile's work:
//   encode: R (tile i+1's 16-B element slots) in flight;  R(i) -> LDS,
//           barrier, issue R(i+1), own 32 elements from LDS -> transposes ->
//           plane dwords, barrier;
//   decode: P (tile i+1's plane dwords) in flight;  P(i) -> transposes ->
//           LDS, issue P(i+1), barrier, coalesced 16-B element stores from
//           LDS, barrier.
// The LDS hand-offs use s_barrier after lgkmcnt(0) only (bf_lds_barrier): a
// full __syncthreads() fence would also wait for the loads in flight.
// 256 MiB, 256 KiB blocks, encode / decode µs (profiles/r05/probe_bshuf_all_*):
// typesize 1 104 / 107 -> 88 / 96, 2 107 / 105 -> 90 / 96, 4 115 / 108 ->
// 90 / 89, 8 135 / 100 -> 96 / 95.
// Not faster: an opaque per-tile plane stride (no hoisted SGPR offsets) cut
// decode to 127 / 181 VGPRs for ES 4 / 8 (from 188 / 255+98 AGPRs, one wave
// per SIMD), yet ts8 decode stayed at 96 us and ts4 rose 88 -> 92 us
// (profiles/r05/probe_bshuf_regtrim.jsonl).
// ---------------------------------------------------------------------------
MC_DEV void bf_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int ES, bool FWD>
__global__ __launch_bounds__(MC_BLOCK) void k_bitshuffle_pipe(const uint8_t *__restrict__ src,
                                                              uint8_t *__restrict__ dst, size_t blocksize,
                                                              size_t nfull) {
  constexpr int SLOTS = 2 * ES;  // 16-B slots per thread
  __shared__ __attribute__((aligned(16))) mc_u32x4 lds[SLOTS * MC_BLOCK];
  const size_t E = blocksize / ES, ng = E / 8, pstride = E / 8;
  const size_t tpb = (ng + BF_GROUPS - 1) / BF_GROUPS;  // tiles per block
  const size_t ntiles = nfull * tpb;
  const int t = threadIdx.x;
  // tile -> (block, first group, groups): full tiles except a block's last
  auto tile = [&](size_t i, size_t &blk, size_t &gw, int &nthr) {
    blk = i / tpb;
    gw = (i - blk * tpb) * BF_GROUPS;
    const size_t gcount = ng - gw < (size_t)BF_GROUPS ? ng - gw : BF_GROUPS;  // multiple of 4
    nthr = (int)(gcount / BF_GPT);
  };
  size_t i = blockIdx.x;
  if (i >= ntiles) return;
  size_t blk, gw;
  int nthr;
  tile(i, blk, gw, nthr);
  if (FWD) {
    mc_u32x4 R[SLOTS];
    auto load = [&](size_t b, size_t g, int nt) {
      const uint8_t *s = src + b * blocksize + g * 8 * ES;
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {
        const int q = t + k * MC_BLOCK;
        if (q < nt * SLOTS) R[k] = mc_ld16<true>(s + 16 * (size_t)q);
      }
    };
    load(blk, gw, nthr);
    for (;;) {
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {
        const int q = t + k * MC_BLOCK;
        if (q < nthr * SLOTS) lds[bf_slot<ES>(q / SLOTS, q % SLOTS)] = R[k];
      }
      bf_lds_barrier();
      const size_t ni = i + gridDim.x;
      size_t nblk = 0, ngw = 0;
      int nnthr = 0;
      if (ni < ntiles) {
        tile(ni, nblk, ngw, nnthr);
        load(nblk, ngw, nnthr);
      }
      if (t < nthr) {
        uint32_t w[8 * ES];
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) {
          const mc_u32x4 v = lds[bf_slot<ES>(t, k)];
          w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
        }
        uint8_t *pd = dst + blk * blocksize + gw + BF_GPT * (size_t)t;
        if constexpr (ES == 4 || ES == 8) bf_planes_store<ES>(w, pd, pstride);
        else bf_planes_store_small<ES>(w, pd, pstride);
      }
      if (ni >= ntiles) return;
      bf_lds_barrier();  // every thread's LDS reads of tile i are done
      i = ni; blk = nblk; gw = ngw; nthr = nnthr;
    }
  } else {
    uint32_t P[8 * ES];
    auto load = [&](size_t b, size_t g, int nt) {
      if (t >= nt) return;
      const uint8_t *ps = src + b * blocksize + g + BF_GPT * (size_t)t;
#pragma unroll
      for (int p = 0; p < 8 * ES; ++p)
        P[p] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(ps + (size_t)p * pstride));
    };
    load(blk, gw, nthr);
    for (;;) {
      if (t < nthr) {
        uint32_t w[8 * ES];
        if constexpr (ES == 4 || ES == 8) {
#pragma unroll
          for (int h = 0; h < ES / 4; ++h) {
            uint32_t a[32];
#pragma unroll
            for (int p = 0; p < 32; ++p) a[p] = P[32 * h + p];
            tr32x32(a);
#pragma unroll
            for (int e = 0; e < 32; ++e) w[(ES / 4) * e + h] = a[e];
          }
        } else {
          bf_elems_small<ES>(P, w);
        }
#pragma unroll
        for (int k = 0; k < SLOTS; ++k)
          lds[bf_slot<ES>(t, k)] = mc_u32x4{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
      }
      const size_t ni = i + gridDim.x;
      size_t nblk = 0, ngw = 0;
      int nnthr = 0;
      if (ni < ntiles) {
        tile(ni, nblk, ngw, nnthr);
        load(nblk, ngw, nnthr);
      }
      bf_lds_barrier();
      uint8_t *d = dst + blk * blocksize + gw * 8 * ES;
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) {
        const int q = t + k * MC_BLOCK;
        if (q < nthr * SLOTS) mc_st16<true>(d + 16 * (size_t)q, lds[bf_slot<ES>(q / SLOTS, q % SLOTS)]);
      }
      if (ni >= ntiles) return;
      bf_lds_barrier();  // the stores' LDS reads are done before the next tile's writes
      i = ni; blk = nblk; gw = ngw; nthr = nnthr;
    }
  }
}

// persistent grid: workgroups per CU as the LDS image allows (8 / 16 / 32 /
// 64 KiB for ES = 1 / 2 / 4 / 8, of 160 KiB; at most 8 of 4 waves)
inline unsigned bf_pipe_grid(int es, size_t ntiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
    else
      cus = 256;
  }
  const size_t g = (size_t)cus * (es == 8 ? 2 : es == 4 ? 4 : 8);
  return (unsigned)(ntiles < g ? ntiles : g);
}

template <int ES>
void launch_bitshuffle_fast(const uint8_t *s, uint8_t *d, size_t nfull, size_t blocksize, bool fwd,
                            hipStream_t st) {
  const size_t ng = blocksize / ES / 8;
  const size_t ntiles = nfull * ((ng + BF_GROUPS - 1) / BF_GROUPS);
  const unsigned g = bf_pipe_grid(ES, ntiles);
  if (fwd) k_bitshuffle_pipe<ES, true><<<g, MC_BLOCK, 0, st>>>(s, d, blocksize, nfull);
  else k_bitshuffle_pipe<ES, false><<<g, MC_BLOCK, 0, st>>>(s, d, blocksize, nfull);
}

inline int launch_bitshuffle_generic(const uint8_t *s, uint8_t *d, size_t nbytes, size_t typesize,
                                     size_t blocksize, bool fwd, hipStream_t st) {
  const size_t nblocks = (nbytes + blocksize - 1) / blocksize;
  const unsigned G = groups_per_wg(typesize);
  const size_t per_wg = (size_t)G * 8 * typesize;
  const size_t span = blocksize < nbytes ? blocksize : nbytes;
  const size_t tiles = (span + per_wg - 1) / per_wg;  // workgroups per block
  if (tiles > 65535 || nblocks > 0x7fffffffu) return MC_EINVAL;
  const dim3 grid((unsigned)nblocks, (unsigned)tiles);
  if (fwd) k_bitshuffle<true><<<grid, MC_BLOCK, 0, st>>>(s, d, nbytes, (unsigned)typesize, blocksize, G);
  else k_bitshuffle<false><<<grid, MC_BLOCK, 0, st>>>(s, d, nbytes, (unsigned)typesize, blocksize, G);
  return mc_last_launch();
}

}  // namespace

extern "C" {

int mc_blosc_filter(const void *src, void *dst, size_t nbytes, size_t typesize, size_t blocksize,
                    int mode, int forward, mc_stream_t stream) {
  if (nbytes == 0) return MC_OK;
  if (!src || !dst || typesize < 1 || typesize > 255 || blocksize < 1) return MC_EINVAL;
  if (mode != MC_BLOSC_NOSHUFFLE && mode != MC_BLOSC_SHUFFLE && mode != MC_BLOSC_BITSHUFFLE)
    return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  if (mode == MC_BLOSC_NOSHUFFLE || (mode == MC_BLOSC_SHUFFLE && typesize == 1))
    return mc_copy_rows_impl(s, nbytes, d, nbytes, nbytes, 1, st);
  if (mode == MC_BLOSC_SHUFFLE) {
    // full blocks as one batch on the Shuffle kernels, then the last block
    const size_t full = nbytes / blocksize, body = blocksize / typesize * typesize;
    int rc = MC_OK;
    if (full) {
      rc = forward ? mc_shuffle_batch(s, blocksize, d, blocksize, full, body, typesize, stream)
                   : mc_unshuffle_batch(s, blocksize, d, blocksize, full, body, typesize, stream);
      if (rc != MC_OK) return rc;
      if (body < blocksize)  // trailing bytes of every full block
        rc = mc_copy_rows_impl(s + body, blocksize, d + body, blocksize, blocksize - body, full, st);
      if (rc != MC_OK) return rc;
    }
    const size_t last = nbytes - full * blocksize;
    if (last) {
      const size_t lb = last / typesize * typesize;
      const uint8_t *ls = s + full * blocksize;
      uint8_t *ld = d + full * blocksize;
      if (lb) {
        rc = forward ? mc_shuffle(ls, ld, lb, typesize, stream) : mc_unshuffle(ls, ld, lb, typesize, stream);
        if (rc != MC_OK) return rc;
      }
      if (lb < last)
        rc = mc_copy_rows_impl(ls + lb, last - lb, ld + lb, last - lb, last - lb, 1, st);
    }
    return rc;
  }
  // bit-shuffle: full blocks on the fast kernel when the layout allows it,
  // the rest (and every other typesize) on the generic one
  const bool fwd = forward != 0;
  const size_t nfull = nbytes / blocksize;
  const bool fast_ts = typesize == 1 || typesize == 2 || typesize == 4 || typesize == 8;
  const bool fast = fast_ts && nfull > 0 && blocksize % (32 * typesize) == 0 &&
                    ((uintptr_t)s & 15) == 0 && ((uintptr_t)d & 15) == 0;
  if (!fast) return launch_bitshuffle_generic(s, d, nbytes, typesize, blocksize, fwd, st);
  switch (typesize) {
    case 1: launch_bitshuffle_fast<1>(s, d, nfull, blocksize, fwd, st); break;
    case 2: launch_bitshuffle_fast<2>(s, d, nfull, blocksize, fwd, st); break;
    case 4: launch_bitshuffle_fast<4>(s, d, nfull, blocksize, fwd, st); break;
    default: launch_bitshuffle_fast<8>(s, d, nfull, blocksize, fwd, st); break;
  }
  const int rc = mc_last_launch();
  if (rc != MC_OK || nbytes == nfull * blocksize) return rc;
  const size_t off = nfull * blocksize;
  return launch_bitshuffle_generic(s + off, d + off, nbytes - off, typesize, blocksize, fwd, st);
}

}  // extern "C"
