// mc_checksum.hip -- the Checksum32 family (checksum32.py:45-209): CRC32
// (zlib.crc32), CRC32C (crc32c / google_crc32c), Adler32 (zlib.adler32) and
// JenkinsLookup3 (jenkins.pyx:93-325), one checksum per chunk over batches of
// chunks, optionally fused with the payload copy of Checksum32.encode.
//
// CRC32 / CRC32C (reflected polynomials 0xEDB88320 / 0x82F63B78).  With the
// raw register update raw(c, D) (no pre/post inversion) the CRC is linear over
// GF(2):  raw(c, D) = c * x^(8|D|) xor raw(0, D)  and  raw(0, zeros ++ D) =
// raw(0, D), and zlib's crc32(D, value) = ~raw(~value, D).  A workgroup owns a
// tile of K * 4096 bytes; lane l reads the 16-B vectors at l*16 + k*4096
// (every load instruction of the wave covers 1 KiB contiguously) and runs
//     acc = raw(acc, v ++ zeros(4080))
// with one slicing-by-16 lookup set whose 16 tables already include the
// 4080-byte shift (V[m][b] = raw(0, byte b ++ zeros(15 - m + 4080))): 16 LDS
// lookups per 16 bytes.  Lane l's accumulator then stands 16*l bytes past the
// tile end; multiplying by x^(-128 l) (x is invertible mod P) aligns every
// lane, and the lanes' values XOR together into the tile's raw CRC.  A
// per-chunk finalize combines tiles with Horner steps by x^(8 * tile bytes)
// and undoes the zero padding of the last tile with x^(-8 * pad).  Bytes past
// the chunk end are read as zeros, so all loads stay vector loads.
//
// Adler32: a = a0 + S1, b = b0 + n*a0 + S2 (mod 65521) with S1 = sum d_i and
// S2 = sum (n - i) d_i -- absolute weights, so it is a plain parallel
// reduction exactly like Fletcher32 (mc_fletcher.hip); byte sums per dword
// come from v_dot4_u32_u8.
//
// JenkinsLookup3 (Bob Jenkins' hashlittle as restated by HDF5) is a serial
// chain of 12-byte mixing rounds with no algebraic shortcut: one thread per
// chunk, so a batch of chunks runs in parallel and a single chunk runs at
// single-thread speed (documented in DESIGN.md).
#include "mc_checksum.h"

#include <stdlib.h>

namespace {
using namespace mcck;

template <int KIND, int K>
__global__ __launch_bounds__(MC_BLOCK) void k_ck_finalize(
    const CrcFin fin, const uint32_t *__restrict__ partials, size_t tiles_per_chunk, size_t n, uint32_t init,
    uint32_t *__restrict__ out, uint8_t *__restrict__ footer, size_t footer_stride,
    const uint8_t *__restrict__ stored, size_t stored_stride, uint32_t *__restrict__ stored_out) {
  ck_finish_chunk<KIND, K, false>(fin, partials, tiles_per_chunk, n, init, out, footer, footer_stride, stored,
                                  stored_stride, stored_out, blockIdx.x);
}

MC_DEV void adler_arrive_finish(uint32_t a1, uint32_t a2, size_t n, const uint8_t *src, size_t src_stride,
                                const struct CkFinish &fx);

template <int KIND, int K, bool COPY, int ALS, int ALD, bool FUSED>
__global__ __launch_bounds__(MC_BLOCK) void k_ck_tiles(
    const uint8_t *__restrict__ src, size_t src_stride, uint8_t *__restrict__ dst,
    size_t dst_stride, size_t n, size_t tiles_per_chunk, size_t total_tiles,
    uint32_t *__restrict__ partials, const CrcFin fin, const CkFinish fx) {
  constexpr bool CRC = KIND != K_ADLER;
  __shared__ uint32_t V[CRC ? 16 * 256 : 1];
  __shared__ uint64_t red[2][MC_BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t g = 0;
  if constexpr (CRC) {
    const mc_u32x4 *tv = reinterpret_cast<const mc_u32x4 *>(&crc_consts<KIND>().v[0][0]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      reinterpret_cast<mc_u32x4 *>(V)[threadIdx.x + i * MC_BLOCK] = tv[threadIdx.x + i * MC_BLOCK];
    g = crc_consts<KIND>().g[threadIdx.x];
    __syncthreads();
  }
  uint32_t adl1 = 0, adl2 = 0;  // FUSED Adler32: the block's (S1, S2) mod P (thread 0)
  for (size_t tile = blockIdx.x; tile < total_tiles; tile += gridDim.x) {
    const size_t c = tile / tiles_per_chunk;
    const size_t t = tile - c * tiles_per_chunk;
    const uint8_t *s = src + c * src_stride;
    const size_t base = t * (size_t)(K * STEP) + 16 * (size_t)threadIdx.x;
    // every tile but a chunk's last lies wholly inside the chunk: plain
    // vector loads / stores with no per-vector bounds checks (tile-uniform branch)
    const bool full = (t + 1) * (size_t)(K * STEP) <= n;
    mc_u32x4 v[K];
    if (full) {
#pragma unroll
      for (int k = 0; k < K; ++k) v[k] = ld_vec<ALS>(s + base + (size_t)k * STEP);
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const size_t pos = base + (size_t)k * STEP;
        v[k] = pos < n ? ld_masked<ALS>(s, pos, n) : mc_u32x4{0, 0, 0, 0};
      }
    }
    if constexpr (COPY) {
      uint8_t *d = dst + c * dst_stride;
      if (full) {
#pragma unroll
        for (int k = 0; k < K; ++k) st_vec<ALD>(d + base + (size_t)k * STEP, v[k]);
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const size_t pos = base + (size_t)k * STEP;
          if (pos < n) st_masked<ALD>(d, pos, n, v[k]);
        }
      }
    }
    if constexpr (CRC) {
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) acc = slice16(V, acc, v[k]);
      acc = wave_xor(gf_mul(acc, g, crc_poly<KIND>()));
      if (lane == 0) red[0][wave] = acc;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t r = 0;
        for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= (uint32_t)red[0][w];
        if constexpr (FUSED) __hip_atomic_store(&partials[tile], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else partials[tile] = r;
      }
    } else {
      uint64_t s1 = 0, s2a = 0, s2b = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const size_t pos = base + (size_t)k * STEP;
        const mc_u32x4 x = v[k];
        const uint32_t a0 = __builtin_amdgcn_udot4(x.x, 0x01010101u, 0u, false);
        const uint32_t a1 = __builtin_amdgcn_udot4(x.y, 0x01010101u, 0u, false);
        const uint32_t a2 = __builtin_amdgcn_udot4(x.z, 0x01010101u, 0u, false);
        const uint32_t a3 = __builtin_amdgcn_udot4(x.w, 0x01010101u, 0u, false);
        uint32_t b = __builtin_amdgcn_udot4(x.x, 0x03020100u, 0u, false);
        b = __builtin_amdgcn_udot4(x.y, 0x07060504u, b, false);
        b = __builtin_amdgcn_udot4(x.z, 0x0b0a0908u, b, false);
        b = __builtin_amdgcn_udot4(x.w, 0x0f0e0d0cu, b, false);
        const uint32_t a = a0 + a1 + a2 + a3;
        // weight of the vector's first byte: n - pos (mod P); bytes >= n are 0
        const uint32_t cw = pos < n ? (uint32_t)((n - pos) % ADLER_P) + ADLER_P : 0u;
        s1 += a;
        s2a += (uint64_t)cw * a;
        s2b += b;
      }
      const uint64_t r1 = wave_sum(s1 % ADLER_P);
      const uint64_t r2 = wave_sum((s2a % ADLER_P + ADLER_P - s2b % ADLER_P) % ADLER_P);
      if (lane == 0) {
        red[0][wave] = r1;
        red[1][wave] = r2;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        uint64_t x = 0, y = 0;
        for (int w = 0; w < MC_BLOCK / 64; ++w) {
          x += red[0][w];
          y += red[1][w];
        }
        if constexpr (FUSED) {
          adl1 = (uint32_t)((adl1 + x) % ADLER_P);
          adl2 = (uint32_t)((adl2 + y) % ADLER_P);
        } else {
          partials[2 * tile] = (uint32_t)(x % ADLER_P);
          partials[2 * tile + 1] = (uint32_t)(y % ADLER_P);
        }
      }
    }
    __syncthreads();  // red[] is reused by the next tile
  }
  if constexpr (FUSED && KIND == K_ADLER) {
    if (threadIdx.x == 0) adler_arrive_finish(adl1, adl2, n, src, src_stride, fx);
    return;
  }
  if constexpr (FUSED) ck_fused_tail<KIND, K>(fin, partials, tiles_per_chunk, n, src_stride, fx);
}


MC_DEV void adler_arrive_finish(uint32_t a1, uint32_t a2, size_t n, const uint8_t *src, size_t src_stride,
                                const CkFinish &fx) {
  (void)src;
  (void)src_stride;
  const unsigned sh = mc_arrival_shard(blockIdx.x);
  unsigned long long *w = reinterpret_cast<unsigned long long *>(fx.ticket + MC_ARRIVAL_LINE * sh);
  const unsigned long long old =
      atomicAdd(w, ((unsigned long long)a2 << 32) | ((unsigned long long)a1 << 8) | 1ull);
  if ((old & 0xffu) + 1u != mc_arrival_per(sh, gridDim.x)) return;
  *w = 0;  // every arrival of this shard is in
  const uint32_t s1 = (uint32_t)((((old >> 8) & 0xffffffu) + a1) % ADLER_P);
  const uint32_t s2 = (uint32_t)((((old >> 32) & 0xffffffu) + a2) % ADLER_P);
  unsigned long long *t = reinterpret_cast<unsigned long long *>(fx.ticket + MC_ARRIVAL_LINE * MC_ARRIVAL_SHARDS);
  const unsigned long long top =
      atomicAdd(t, ((unsigned long long)s2 << 32) | ((unsigned long long)s1 << 8) | 1ull);
  if ((top & 0xffu) + 1u != mc_arrival_nshards(gridDim.x)) return;
  *t = 0;
  uint64_t x = (((top >> 8) & 0xffffffu) + s1) % ADLER_P;
  uint64_t y = (((top >> 32) & 0xffffffu) + s2) % ADLER_P;
  // head: the tiles started at the 4 stored bytes (byte j weighted n - j); take them out
  for (uint32_t j = 0; j < fx.head; ++j) {
    const uint64_t dj = fx.stored[j];
    x = (x + ADLER_P - dj) % ADLER_P;
    y = (y + ADLER_P - (uint64_t)((n - j) % ADLER_P) * dj % ADLER_P) % ADLER_P;
  }
  const size_t np = n - fx.head;  // payload bytes
  // zlib.adler32(data, value): a0 = value & 0xffff, b0 = value >> 16
  const uint64_t a0 = fx.init & 0xffffu, b0 = fx.init >> 16;
  const uint64_t a = (a0 + x) % ADLER_P;
  const uint64_t b = (b0 + (np % ADLER_P) * a0 + y) % ADLER_P;
  const uint32_t result = (uint32_t)((b << 16) | a);
  if (fx.stored_out) fx.stored_out[0] = load_le32(fx.stored);
  if (fx.out) fx.out[0] = result;
  if (fx.footer) store_le32(fx.footer, result);
  mc_publish_verdict_seq(fx.out, fx.seq);
}

// ---------------------------------------------------------------------------
// JenkinsLookup3 (jenkins.pyx:93-325): one thread per chunk over the virtual
// stream prefix ++ chunk.
// ---------------------------------------------------------------------------
MC_DEV uint32_t jrot(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

MC_DEV void jmix(uint32_t &a, uint32_t &b, uint32_t &c) {  // jenkins.pyx:264-325
  a -= c; a ^= jrot(c, 4);  c += b;
  b -= a; b ^= jrot(a, 6);  a += c;
  c -= b; c ^= jrot(b, 8);  b += a;
  a -= c; a ^= jrot(c, 16); c += b;
  b -= a; b ^= jrot(a, 19); a += c;
  c -= b; c ^= jrot(b, 4);  b += a;
}

MC_DEV uint32_t jfinal(uint32_t a, uint32_t b, uint32_t c) {  // jenkins.pyx:221-259
  c ^= b; c -= jrot(b, 14);
  a ^= c; a -= jrot(c, 11);
  b ^= a; b -= jrot(a, 25);
  c ^= b; c -= jrot(b, 16);
  a ^= c; a -= jrot(c, 4);
  b ^= a; b -= jrot(a, 14);
  c ^= b; c -= jrot(b, 24);
  return c;
}

MC_DEV uint32_t jbyte(const uint8_t *pre, size_t plen, const uint8_t *s, size_t i) {
  return i < plen ? pre[i] : s[i - plen];
}

__global__ __launch_bounds__(64) void k_jenkins(const uint8_t *__restrict__ src, size_t src_stride,
                                                size_t nchunks, size_t n, uint32_t init,
                                                const uint8_t *__restrict__ prefix, size_t plen,
                                                uint32_t *__restrict__ out,
                                                uint8_t *__restrict__ footer,
                                                size_t footer_stride,
                                                const uint8_t *__restrict__ stored,
                                                uint32_t *__restrict__ stored_out) {
  const size_t ci = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= nchunks) return;
  if (stored_out) stored_out[ci] = load_le32(stored + ci * src_stride);
  const uint8_t *s = src + ci * src_stride;
  const size_t L = plen + n;
  uint32_t a, b, c;
  a = b = c = 0xdeadbeefu + (uint32_t)L + init;
  if (L > 0) {
    const size_t nb = (L - 1) / 12;  // full mixing blocks ("while length > 12")
    size_t blk = 0;
    if (plen == 0 && ((uintptr_t)s & 15) == 0) {
      // 16 blocks (192 B = 12 x 16-B loads) per group in a ring of JR groups:
      // group g + JR - 1 is loaded while group g mixes.  A group's 16 mixes
      // (~1100 cycles of dependent ALU work) are shorter than a load's
      // latency, so one group ahead left the chain waiting on memory: one
      // 16 MiB chunk 98 -> 73 ms, 2048 x 1 MiB 300 -> 392 GB/s
      // (tools/probe_jenkins.py).  A second wave prefetching the chunk into
      // L2 ahead of the chain measured no further gain (74.9 ms): the chain's
      // ~125 cycles per 12-B block are its dependent mix operations
      constexpr size_t G = 16;
      constexpr int JR = 4;
      const mc_u32x4 *v4 = reinterpret_cast<const mc_u32x4 *>(s);
      const size_t ng = nb / G;
      mc_u32x4 ring[JR][12];
#pragma unroll
      for (int r = 0; r + 1 < JR; ++r)
        if ((size_t)r < ng) {
#pragma unroll
          for (int j = 0; j < 12; ++j) ring[r][j] = v4[12 * r + j];
        }
      for (size_t gi = 0; gi < ng; gi += JR) {
#pragma unroll
        for (int r = 0; r < JR; ++r) {
          const size_t g = gi + r;
          if (g >= ng) break;
          if (g + JR - 1 < ng) {
#pragma unroll
            for (int j = 0; j < 12; ++j) ring[(r + JR - 1) % JR][j] = v4[12 * (g + JR - 1) + j];
          }
          uint32_t q[48];
#pragma unroll
          for (int j = 0; j < 12; ++j) {
            q[4 * j] = ring[r][j].x; q[4 * j + 1] = ring[r][j].y;
            q[4 * j + 2] = ring[r][j].z; q[4 * j + 3] = ring[r][j].w;
          }
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            a += q[3 * k];
            b += q[3 * k + 1];
            c += q[3 * k + 2];
            jmix(a, b, c);
          }
        }
      }
      blk = ng * G;
      const uint32_t *w = reinterpret_cast<const uint32_t *>(s);
      for (; blk < nb; ++blk) {
        a += w[3 * blk];
        b += w[3 * blk + 1];
        c += w[3 * blk + 2];
        jmix(a, b, c);
      }
    } else if (plen == 0 && ((uintptr_t)s & 3) == 0) {
      const uint32_t *w = reinterpret_cast<const uint32_t *>(s);
      for (; blk < nb; ++blk) {
        a += w[3 * blk];
        b += w[3 * blk + 1];
        c += w[3 * blk + 2];
        jmix(a, b, c);
      }
    } else {
      for (; blk < nb; ++blk) {
        uint32_t q[3] = {0, 0, 0};
        for (int j = 0; j < 12; ++j) q[j >> 2] += jbyte(prefix, plen, s, 12 * blk + j) << (8 * (j & 3));
        a += q[0];
        b += q[1];
        c += q[2];
        jmix(a, b, c);
      }
    }
    // last block: 1..12 bytes (the fall-through switch of jenkins.pyx:167-214)
    const size_t r = L - 12 * nb;
    uint32_t q[3] = {0, 0, 0};
    for (size_t j = 0; j < r; ++j) q[j >> 2] += jbyte(prefix, plen, s, 12 * nb + j) << (8 * (j & 3));
    a += q[0];
    b += q[1];
    c += q[2];
    c = jfinal(a, b, c);
  }
  if (out) out[ci] = c;
  if (footer) store_le32(footer + ci * footer_stride, c);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Schedule (mc_sched.h): ck_k / ck_kcopy = tile size in STEP units for
// chunks of >= 64 KiB (4, 8 or 16) without / with the fused payload copy,
// ck_grid / ck_grid_copy = persistent grid caps.  Defaults
// from the sweep on 64 x 4 MiB: the checksum alone is best with
// 64 KiB tiles, the copying passes (encode, decode) with 32 KiB tiles and
// 1024 workgroups (CRC32 decode 139 -> 120 us).
inline int ck_kbig() {
  const int e = mc_sched.ck_k;
  return (e == 4 || e == 8 || e == 16) ? e : 16;
}
// the one-launch verify's tile: 32 KiB.  CRC (K = 8: 159 VGPRs, three waves
// per SIMD) on one round of 768 workgroups, against 64 KiB tiles on 512: 256
// MiB CRC32 / CRC32C 46.0 / 45.6 us back to back (47.8 / 47.4 single) against
// 47.8 / 46.6 (48.9 / 48.0); 16 KiB tiles 52-66 us (tools/probe_ck_verify_grid6.py
// CK_KSWEEP=1, profiles/r06/probe_crc_verify_k.jsonl).  Adler32 on 1024
// workgroups: 44.6 us back to back (46.9 single) against 47.3 (51.8) for 64
// KiB tiles on 2048 (CK_ADLER=1 CK_KSWEEP=1, probe_adler_verify_k.jsonl)
constexpr int CK_VERIFY_K = 8;
constexpr unsigned ADLER_VERIFY_GRID = 1024;
inline int ck_k_verify(size_t n) {
  const int e = mc_sched.ck_k;
  return n < (size_t)16 * STEP ? 1 : (e == 4 || e == 8 || e == 16) ? e : CK_VERIFY_K;
}
inline int ck_kcopy() {
  const int e = mc_sched.ck_kcopy;
  return (e == 4 || e == 8 || e == 16) ? e : 8;
}
// persistent-grid caps (ck_grid / ck_grid_copy).  The
// checksum-only CRC kernels run fastest with one tile per workgroup (no
// cap): one 256 MiB CRC32 verify 69.3 us at 2048 workgroups, 64.7 at 4096,
// 63.9 at 8192 = every tile; Adler32 is best at 2048 (48.3 us, 50.1 at
// 4096-8192) (tools/probe_adler_verify.py, profiles/r02/probe_ck_verify_grid.jsonl)
inline unsigned ck_grid_cap(bool copy, bool crc) {
  const int g = mc_sched.ck_grid;
  const unsigned gc = mc_sched.ck_grid_copy > 0 ? (unsigned)mc_sched.ck_grid_copy : 1024u;
  if (copy) return gc;
  if (g > 0) return (unsigned)g;
  return crc ? 0xffffffffu : 2048u;
}

// the bit-sliced CRC kernel's grid: ck_grid / ck_grid_copy when set, else
// 2048 workgroups for the checksum-only passes (two resident per CU, so four
// rounds of two tiles each: 1-2 us faster than one round of 512 persistent
// workgroups for the 256 MiB verify, profiles/r03/probe_crc_bs.jsonl) and the
// copy passes' 1024
inline unsigned ck_grid_cap_bs(bool copy) {
  const int g = copy ? mc_sched.ck_grid_copy : mc_sched.ck_grid;
  return g > 0 ? (unsigned)g : 2048u;
}

// the bit-sliced kernel's grid; its one-launch finish (ck_ride_arrive) takes
// at most CK_RIDE_MAX_GRID workgroups.  The one-launch verify runs one round
// of resident workgroups (three per CU with CK_VERIFY_K's registers, 768):
// with the sums riding the arrival atomics, one round beat four (64 KiB
// tiles: 48.6 / 48.7 us per single launch on 512 workgroups against 50.3 /
// 49.6 on 2048; tools/probe_ck_verify_grid6.py,
// profiles/r06/probe_ck_verify_grid6.jsonl)
constexpr unsigned CK_VERIFY_GRID = 768;
inline unsigned ck_bs_grid(size_t total, bool copy, bool fused) {
  unsigned cap = ck_grid_cap_bs(copy);
  if (fused && !copy && mc_sched.ck_grid <= 0) cap = CK_VERIFY_GRID;
  if (fused && cap > CK_RIDE_MAX_GRID) cap = CK_RIDE_MAX_GRID;
  return (unsigned)(total < cap ? total : cap);
}

// tile size (in STEP units) for a chunk: K = 1 below 64 KiB
inline int ck_k(size_t n, bool copy) {
  return n < (size_t)16 * STEP ? 1 : copy ? ck_kcopy() : ck_kbig();
}
// the workspace covers every pass
inline int ck_k_ws(size_t n) {
  const int a = ck_k(n, false), b = ck_k(n, true), c = ck_k_verify(n);
  const int m = a < b ? a : b;
  return m < c ? m : c;
}
inline size_t ck_tiles(size_t n, int K) {
  const size_t tb = (size_t)K * STEP;
  return n ? (n + tb - 1) / tb : 1;
}
inline int align_class(const void *p, size_t stride, size_t nchunks) {
  const uintptr_t a = (uintptr_t)p | (nchunks > 1 ? stride : 0);
  return (a & 15) == 0 ? 2 : (a & 3) == 0 ? 1 : 0;
}

template <int KIND, int K, bool COPY, int ALS, int ALD>
void launch_tiles(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t n, size_t tpc,
                  size_t total, uint32_t *parts, const CrcFin &fin, const CkFinish *fx, hipStream_t st) {
  unsigned cap = ck_grid_cap(COPY, KIND != K_ADLER);
  if (fx && KIND == K_ADLER && !COPY && mc_sched.ck_grid <= 0) cap = ADLER_VERIFY_GRID;  // (CK_VERIFY_K)
  const unsigned grid = (unsigned)(total < cap ? total : cap);
  if (fx) {  // one chunk: the last block finishes it in this launch (verify, or encode with its copy)
    const unsigned fg = KIND == K_ADLER && grid > ADLER_MAX_GRID ? ADLER_MAX_GRID : grid;
    k_ck_tiles<KIND, K, COPY, ALS, ALD, true><<<fg, MC_BLOCK, 0, st>>>(s, ss, d, ds, n, tpc, total, parts,
                                                                       fin, *fx);
    return;
  }
  k_ck_tiles<KIND, K, COPY, ALS, ALD, false><<<grid, MC_BLOCK, 0, st>>>(s, ss, d, ds, n, tpc, total, parts, fin,
                                                                        CkFinish{});
}

template <int KIND, int K>
void dispatch_tiles(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t nchunks, size_t n,
                    size_t tpc, uint32_t *parts, const CrcFin &fin, const CkFinish *fx, hipStream_t st) {
  const size_t total = tpc * nchunks;
  const int als = align_class(s, ss, nchunks);
  if (KIND != K_ADLER && K >= 4 && !mc_sched.crc_lds) {  // bit-sliced fold, persistent pipelined grid
    const unsigned grid = ck_bs_grid(total, d != nullptr, fx != nullptr);
    launch_crc_bs(KIND, K, als, d ? align_class(d, ds, nchunks) : 2, s, ss, d, ds, n, tpc, total, parts, fin, fx,
                  grid, st);
    return;
  }
  if (!d) {
    if (als == 2) launch_tiles<KIND, K, false, 2, 2>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
    else if (als == 1) launch_tiles<KIND, K, false, 1, 1>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
    else launch_tiles<KIND, K, false, 0, 0>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
    return;
  }
  const int ald = align_class(d, ds, nchunks);
  if (als == 2 && ald == 2) launch_tiles<KIND, K, true, 2, 2>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
  else if (als == 1 && ald == 2) launch_tiles<KIND, K, true, 1, 2>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
  else if (als == 2 && ald == 1) launch_tiles<KIND, K, true, 2, 1>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
  else if (als >= 1 && ald >= 1) launch_tiles<KIND, K, true, 1, 1>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
  else launch_tiles<KIND, K, true, 0, 0>(s, ss, d, ds, n, tpc, total, parts, fin, fx, st);
}

// host: x^(2^k) / x^(-2^k) tables (64 squarings, once per polynomial)
struct HostPow {
  uint32_t x2n[64], x2n_inv[64];
  explicit HostPow(uint32_t poly) {
    x2n[0] = GF_X;
    x2n_inv[0] = (poly << 1) | 1u;
    for (int k = 1; k < 64; ++k) {
      x2n[k] = gf_mul(x2n[k - 1], x2n[k - 1], poly);
      x2n_inv[k] = gf_mul(x2n_inv[k - 1], x2n_inv[k - 1], poly);
    }
  }
  static uint32_t pw(const uint32_t (&t)[64], uint64_t e, uint32_t poly) {
    uint32_t p = GF_ONE;
    for (int k = 0; e; ++k, e >>= 1)
      if (e & 1) p = gf_mul(p, t[k], poly);
    return p;
  }
};

// n: bytes the tiles cover; np: payload bytes (n - 4 with a head, else n);
// G: the bit-sliced kernel's grid (its one-launch finish)
template <int KIND>
CrcFin crc_fin_build(int K, size_t tpc, size_t n, size_t np, unsigned G) {
  CrcFin f{};
  f.head = n != np;
  if constexpr (KIND != K_ADLER) {
    constexpr uint32_t poly = crc_poly<KIND>();
    static const HostPow hp(poly);
    const uint64_t tb = (uint64_t)K * STEP;
    uint32_t xt[32];  // X^(2^k)
    xt[0] = HostPow::pw(hp.x2n, 8 * tb, poly);
    for (int k = 1; k < 32; ++k) xt[k] = gf_mul(xt[k - 1], xt[k - 1], poly);
    for (int m = 0; m < 32; ++m) f.xb[m] = gf_mul(1u << m, xt[0], poly);
    // tail[t] = X^(tpc - hi(t)), walking t down: each step multiplies by
    // X^(hi(t+1) - hi(t)), one of two exponents (floor / ceil of tpc/256)
    const uint64_t d0 = tpc / MC_BLOCK;
    auto xpow = [&](uint64_t e) {
      uint32_t p = GF_ONE;
      for (int k = 0; e; ++k, e >>= 1)
        if (e & 1) p = gf_mul(p, xt[k], poly);
      return p;
    };
    const uint32_t m0 = xpow(d0), m1 = xpow(d0 + 1);
    f.tail[MC_BLOCK - 1] = GF_ONE;
    for (int t = MC_BLOCK - 2; t >= 0; --t) {
      const uint64_t step = tpc * (t + 2) / MC_BLOCK - tpc * (t + 1) / MC_BLOCK;
      f.tail[t] = step == 0 ? f.tail[t + 1] : gf_mul(f.tail[t + 1], step == d0 ? m0 : m1, poly);
    }
    f.pad = HostPow::pw(hp.x2n_inv, 8 * (tb * tpc - n), poly);
    f.xn = HostPow::pw(hp.x2n, 8 * (uint64_t)np, poly);
    const uint32_t xg = xpow(G);
    for (int m = 0; m < 32; ++m) f.xgb[m] = gf_mul(1u << m, xg, poly);
    f.xh = HostPow::pw(hp.x2n, 8 * (uint64_t)np + 32, poly);
  }
  return f;
}

// the constants of the last call on this thread (a stream of equal-size
// chunks asks for the same ones every time)
template <int KIND>
const CrcFin &crc_fin(int K, size_t tpc, size_t n, size_t np, unsigned G) {
  thread_local struct {
    int K = -1;
    size_t tpc = 0, n = 0, np = 0;
    unsigned G = 0;
    CrcFin f;
  } last;
  if (KIND != K_ADLER && (last.K != K || last.tpc != tpc || last.n != n || last.np != np || last.G != G)) {
    last.f = crc_fin_build<KIND>(K, tpc, n, np, G);
    last.K = K;
    last.tpc = tpc;
    last.n = n;
    last.np = np;
    last.G = G;
  }
  return last.f;
}

template <int KIND>
int run_reduction(const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t nchunks, size_t n,
                  uint32_t init, uint32_t *out, uint8_t *footer, size_t fs, const uint8_t *stored,
                  uint32_t *stored_out, void *ws, size_t ws_bytes, hipStream_t st, uint32_t *ticket,
                  uint32_t seq, uint32_t head) {
  // head = 4: s is the 16-B aligned buffer start, 4 stored bytes before the
  // n payload bytes; the tiles cover all n + 4 (one-launch verify only)
  const size_t np = n;
  n += head;
  // one chunk with a ticket: finish in the tiles launch (ck_finish_chunk)
  const bool fused = ticket && nchunks == 1;
  const int K = fused && !d && (KIND == K_ADLER || !mc_sched.crc_lds) ? ck_k_verify(n) : ck_k(n, d != nullptr);
  const size_t tpc = ck_tiles(n, K);
  const size_t need = tpc * nchunks * (KIND == K_ADLER ? 8 : 4);
  if (!ws || ws_bytes < need) return MC_ENOSPC;
  uint32_t *parts = static_cast<uint32_t *>(ws);
  CkFinish fx{init, seq, head, ticket, out, stored_out, footer, fs, stored, 0};
  const unsigned G = ck_bs_grid(tpc * nchunks, d != nullptr, fused);
  switch (K) {
#define MC_CK_CASE(KK)                                                                         \
  case KK: {                                                                                   \
    const CrcFin &fin = crc_fin<KIND>(KK, tpc, n, np, G);                                      \
    if constexpr (KIND != K_ADLER) fx.c0 = gf_mul(~init, fin.xn, crc_poly<KIND>());            \
    dispatch_tiles<KIND, KK>(s, ss, d, ds, nchunks, n, tpc, parts, fin, fused ? &fx : nullptr, st); \
    if (!fused)                                                                                \
      k_ck_finalize<KIND, KK><<<(unsigned)nchunks, MC_BLOCK, 0, st>>>(                         \
          fin, parts, tpc, n, init, out, footer, fs, stored, ss, stored_out);                  \
    break;                                                                                     \
  }
    MC_CK_CASE(1)
    MC_CK_CASE(4)
    MC_CK_CASE(8)
    MC_CK_CASE(16)
#undef MC_CK_CASE
    default:
      return MC_EINVAL;
  }
  return mc_last_launch();
}

int ck_dispatch(int kind, const uint8_t *s, size_t ss, uint8_t *d, size_t ds, size_t nchunks,
                size_t n, uint32_t init, const uint8_t *prefix, size_t plen, uint32_t *out,
                uint8_t *footer, size_t fs, const uint8_t *stored, uint32_t *stored_out, void *ws,
                size_t ws_bytes, hipStream_t st, uint32_t *ticket = nullptr, uint32_t seq = 0,
                uint32_t head = 0) {
  switch (kind) {
    case MC_CK_CRC32:
      return run_reduction<K_CRC32>(s, ss, d, ds, nchunks, n, init, out, footer, fs, stored, stored_out,
                                    ws, ws_bytes, st, ticket, seq, head);
    case MC_CK_CRC32C:
      return run_reduction<K_CRC32C>(s, ss, d, ds, nchunks, n, init, out, footer, fs, stored, stored_out,
                                     ws, ws_bytes, st, ticket, seq, head);
    case MC_CK_ADLER32:
      return run_reduction<K_ADLER>(s, ss, d, ds, nchunks, n, init, out, footer, fs, stored, stored_out,
                                    ws, ws_bytes, st, ticket, seq, head);
    case MC_CK_JENKINS: {
      if (d && n) {
        const int rc = mc_copy_rows_impl(s, ss, d, ds, n, nchunks, st);
        if (rc != MC_OK) return rc;
      }
      const unsigned grid = (unsigned)((nchunks + 63) / 64);
      k_jenkins<<<grid, 64, 0, st>>>(s, ss, nchunks, n, init, prefix, plen, out, footer, fs, stored,
                                     stored_out);
      return mc_last_launch();
    }
    default:
      return MC_EINVAL;
  }
}

bool valid_kind(int kind) { return kind >= MC_CK_CRC32 && kind <= MC_CK_JENKINS; }

}  // namespace

extern "C" {

size_t mc_checksum32_workspace(int kind, size_t nchunks, size_t chunk_bytes) {
  if (!valid_kind(kind) || kind == MC_CK_JENKINS) return 0;
  // a one-launch verify may tile the stored word with the payload (+ 4)
  const size_t t0 = ck_tiles(chunk_bytes, ck_k_ws(chunk_bytes));
  const size_t t4 = ck_tiles(chunk_bytes + 4, ck_k_ws(chunk_bytes + 4));
  const size_t tpc = t0 > t4 ? t0 : t4;
  return tpc * nchunks * (kind == MC_CK_ADLER32 ? 8 : 4);
}

int mc_checksum32_batch(int kind, const void *src, size_t src_stride, size_t nchunks,
                        size_t chunk_bytes, uint32_t init, const void *prefix, size_t prefix_bytes,
                        uint32_t *out_sums, void *workspace, size_t workspace_bytes,
                        mc_stream_t stream) {
  if (!valid_kind(kind)) return MC_EINVAL;
  if (nchunks == 0) return MC_OK;
  if (!out_sums || (chunk_bytes && !src) || (nchunks > 1 && src_stride < chunk_bytes)) return MC_EINVAL;
  if (prefix_bytes && (kind != MC_CK_JENKINS || !prefix)) return MC_EINVAL;
  if (nchunks > 0x7fffffffu) return MC_EINVAL;
  return ck_dispatch(kind, static_cast<const uint8_t *>(src), src_stride, nullptr, 0, nchunks,
                     chunk_bytes, init, static_cast<const uint8_t *>(prefix), prefix_bytes,
                     out_sums, nullptr, 0, nullptr, nullptr, workspace, workspace_bytes,
                     (hipStream_t)stream);
}

int mc_checksum32_encode_batch(int kind, const void *src, size_t src_stride, void *dst,
                               size_t dst_stride, size_t nchunks, size_t chunk_bytes,
                               uint32_t init, const void *prefix, size_t prefix_bytes,
                               int location, uint32_t *out_sums, void *workspace,
                               size_t workspace_bytes, mc_stream_t stream) {
  if (!valid_kind(kind) || (location != MC_CK_START && location != MC_CK_END)) return MC_EINVAL;
  if (nchunks == 0) return MC_OK;
  if (!dst || (chunk_bytes && !src)) return MC_EINVAL;
  if (nchunks > 1 && (src_stride < chunk_bytes || dst_stride < chunk_bytes + 4)) return MC_EINVAL;
  if (prefix_bytes && (kind != MC_CK_JENKINS || !prefix)) return MC_EINVAL;
  if (nchunks > 0x7fffffffu) return MC_EINVAL;
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint8_t *payload = location == MC_CK_START ? d + 4 : d;
  uint8_t *footer = location == MC_CK_START ? d : d + chunk_bytes;
  return ck_dispatch(kind, static_cast<const uint8_t *>(src), src_stride, payload, dst_stride,
                     nchunks, chunk_bytes, init, static_cast<const uint8_t *>(prefix),
                     prefix_bytes, out_sums, footer, dst_stride, nullptr, nullptr, workspace,
                     workspace_bytes, (hipStream_t)stream);
}

int mc_checksum32_decode_batch(int kind, const void *src, size_t src_stride, void *dst,
                               size_t dst_stride, size_t nchunks, size_t encoded_bytes,
                               uint32_t init, const void *prefix, size_t prefix_bytes,
                               int location, uint32_t *out_sums, uint32_t *out_stored,
                               void *workspace, size_t workspace_bytes, mc_stream_t stream) {
  if (!valid_kind(kind) || (location != MC_CK_START && location != MC_CK_END)) return MC_EINVAL;
  if (nchunks == 0) return MC_OK;
  if (encoded_bytes < 4 || !src || !out_sums || !out_stored) return MC_EINVAL;
  const size_t n = encoded_bytes - 4;
  if (nchunks > 1 && (src_stride < encoded_bytes || (dst && dst_stride < n))) return MC_EINVAL;
  if (prefix_bytes && (kind != MC_CK_JENKINS || !prefix)) return MC_EINVAL;
  if (nchunks > 0x7fffffffu) return MC_EINVAL;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  const uint8_t *payload = location == MC_CK_START ? s + 4 : s;
  const uint8_t *stored = location == MC_CK_START ? s : s + n;
  return ck_dispatch(kind, payload, src_stride, static_cast<uint8_t *>(dst), dst_stride, nchunks, n,
                     init, static_cast<const uint8_t *>(prefix), prefix_bytes, out_sums, nullptr, 0,
                     stored, out_stored, workspace, workspace_bytes, (hipStream_t)stream);
}

// Checksum32.decode's verification of ONE encoded buffer in one launch: the
// checksum's last tile block folds the partials (CRC32 / CRC32C / Adler32;
// Jenkins is one kernel anyway).  out_pair[0] = checksum of the payload,
// out_pair[1] = the stored LE32 value; out_pair may be host-mapped pinned
// memory.  `ticket`: one device word, zero before the first call, left zero
// (keep one per stream); NULL = the two-launch path.
int mc_checksum32_encode_fused(int kind, const void *src, void *dst, size_t chunk_bytes, uint32_t init,
                               const void *prefix, size_t prefix_bytes, int location, uint32_t *out_sum,
                               void *workspace, size_t workspace_bytes, uint32_t *ticket, mc_stream_t stream) {
  if (!ticket || kind == MC_CK_JENKINS)  // Jenkins has no one-launch fold: the batched entry point
    return mc_checksum32_encode_batch(kind, src, chunk_bytes, dst, chunk_bytes + 4, 1, chunk_bytes, init, prefix,
                                      prefix_bytes, location, out_sum, workspace, workspace_bytes, stream);
  if (!valid_kind(kind) || (location != MC_CK_START && location != MC_CK_END)) return MC_EINVAL;
  if (!dst || (chunk_bytes && !src) || (uintptr_t)ticket % 8) return MC_EINVAL;
  if (prefix_bytes) return MC_EINVAL;  // a prefix belongs to Jenkins only
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint8_t *payload = location == MC_CK_START ? d + 4 : d;
  uint8_t *footer = location == MC_CK_START ? d : d + chunk_bytes;
  return ck_dispatch(kind, static_cast<const uint8_t *>(src), 0, payload, 0, 1, chunk_bytes, init, nullptr, 0,
                     out_sum, footer, 0, nullptr, nullptr, workspace, workspace_bytes, (hipStream_t)stream, ticket, 0);
}

int mc_checksum32_verify_fused(int kind, const void *src, size_t encoded_bytes, uint32_t init,
                               const void *prefix, size_t prefix_bytes, int location, uint32_t *out_pair,
                               uint32_t seq, void *workspace, size_t workspace_bytes, uint32_t *ticket,
                               mc_stream_t stream) {
  if (!valid_kind(kind) || (location != MC_CK_START && location != MC_CK_END)) return MC_EINVAL;
  if (encoded_bytes < 4 || !src || !out_pair) return MC_EINVAL;
  // only the one-launch finish of CRC32 / CRC32C / Adler32 publishes `seq`
  if (seq && (!ticket || kind == MC_CK_JENKINS)) return MC_EINVAL;
  if (ticket && (uintptr_t)ticket % 8) return MC_EINVAL;  // 64-bit arrival words (Adler32)
  if (prefix_bytes && (kind != MC_CK_JENKINS || !prefix)) return MC_EINVAL;
  const size_t n = encoded_bytes - 4;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  const uint8_t *payload = location == MC_CK_START ? s + 4 : s;
  const uint8_t *stored = location == MC_CK_START ? s : s + n;
  // location "start" on a 16-B aligned buffer: the payload at +4 would be read
  // with dword-aligned vectors; the one-launch CRC / Adler32 verify instead
  // tiles the whole aligned buffer and removes the stored word's share at its
  // finish (CrcFin::head, adler_arrive_finish)
  if (ticket && location == MC_CK_START && kind != MC_CK_JENKINS && ((uintptr_t)s & 15) == 0 && n >= 16)
    return ck_dispatch(kind, s, encoded_bytes, nullptr, 0, 1, n, init, nullptr, 0, out_pair, nullptr, 0, stored,
                       out_pair + 1, workspace, workspace_bytes, (hipStream_t)stream, ticket, seq, 4);
  return ck_dispatch(kind, payload, encoded_bytes, nullptr, 0, 1, n, init, static_cast<const uint8_t *>(prefix),
                     prefix_bytes, out_pair, nullptr, 0, stored, out_pair + 1, workspace, workspace_bytes,
                     (hipStream_t)stream, ticket, seq);
}

}  // extern "C"
