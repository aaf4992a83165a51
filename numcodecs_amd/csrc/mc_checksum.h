// mc_checksum.h -- device building blocks shared by the Checksum32 kernels
// (mc_checksum.hip: table folds, Adler32, Jenkins, host side; mc_crc_bs.hip:
// the bit-sliced CRC tile kernel), split so the two heavy template sets
// compile in parallel.  Derivations: the header of mc_checksum.hip.
#pragma once
#include "mc_common.h"
#include "mc_crc_bs.h"

namespace mcck {

// ---------------------------------------------------------------------------
// GF(2)[x] mod P in the reflected representation (bit 31 = x^0, bit 0 = x^31)
// ---------------------------------------------------------------------------
constexpr uint32_t POLY_CRC32 = 0xEDB88320u;
constexpr uint32_t POLY_CRC32C = 0x82F63B78u;
constexpr uint32_t GF_ONE = 0x80000000u;  // x^0
constexpr uint32_t GF_X = 0x40000000u;    // x^1

constexpr MC_HD uint32_t gf_mul(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (GF_ONE >> i)) p ^= b;                   // + a_i * b * x^i
    b = (b & 1u) ? ((b >> 1) ^ poly) : (b >> 1);     // b *= x
  }
  return p;
}

constexpr int STEP = MC_BLOCK * 16;  // bytes between a lane's consecutive vectors
constexpr int SHIFT = STEP - 16;     // zero bytes folded into the tables

struct CrcConsts {
  uint32_t v[16][256];  // V[m][b] = raw(0, byte b ++ zeros(15 - m + SHIFT))
  uint32_t g[MC_BLOCK];  // x^(-128 l): moves lane l's accumulator back 16*l bytes
  uint32_t x2n[64];      // x^(2^k)
  uint32_t x2n_inv[64];  // x^(-2^k)
};

constexpr uint32_t xpow_tab(const uint32_t (&tab)[64], uint64_t e, uint32_t poly) {
  uint32_t p = GF_ONE;
  for (int k = 0; e; ++k, e >>= 1)
    if (e & 1) p = gf_mul(p, tab[k], poly);
  return p;
}

constexpr CrcConsts make_crc_consts(uint32_t poly) {
  CrcConsts c{};
  uint32_t t[16][256] = {};
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t r = b;
    for (int k = 0; k < 8; ++k) r = (r & 1u) ? ((r >> 1) ^ poly) : (r >> 1);
    t[0][b] = r;  // raw(0, byte b)
  }
  for (int k = 1; k < 16; ++k)
    for (int b = 0; b < 256; ++b) t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xffu];
  c.x2n[0] = GF_X;
  for (int k = 1; k < 64; ++k) c.x2n[k] = gf_mul(c.x2n[k - 1], c.x2n[k - 1], poly);
  // x * (P(x) - 1)/x = P(x) - 1 = 1 (mod P, mod 2): x^-1 = (P - 1)/x
  c.x2n_inv[0] = (poly << 1) | 1u;
  for (int k = 1; k < 64; ++k) c.x2n_inv[k] = gf_mul(c.x2n_inv[k - 1], c.x2n_inv[k - 1], poly);
  const uint32_t z = xpow_tab(c.x2n, 8ull * SHIFT, poly);
  for (int m = 0; m < 16; ++m) {
    uint32_t basis[8] = {};
    for (int j = 0; j < 8; ++j) basis[j] = gf_mul(t[15 - m][1u << j], z, poly);
    for (int b = 0; b < 256; ++b) {  // raw(0, .) is linear in the byte
      uint32_t r = 0;
      for (int j = 0; j < 8; ++j)
        if (b & (1 << j)) r ^= basis[j];
      c.v[m][b] = r;
    }
  }
  c.g[0] = GF_ONE;
  for (int l = 1; l < MC_BLOCK; ++l) c.g[l] = gf_mul(c.g[l - 1], c.x2n_inv[7], poly);
  return c;
}

static_assert(gf_mul(GF_X, (POLY_CRC32 << 1) | 1u, POLY_CRC32) == GF_ONE, "x^-1 (CRC32)");
static_assert(gf_mul(GF_X, (POLY_CRC32C << 1) | 1u, POLY_CRC32C) == GF_ONE, "x^-1 (CRC32C)");

static __constant__ const CrcConsts kCrc32 = make_crc_consts(POLY_CRC32);
static __constant__ const CrcConsts kCrc32c = make_crc_consts(POLY_CRC32C);

enum Kind { K_CRC32 = MC_CK_CRC32, K_CRC32C = MC_CK_CRC32C, K_ADLER = MC_CK_ADLER32 };

template <int KIND>
MC_DEV const CrcConsts &crc_consts() {
  if constexpr (KIND == K_CRC32C) return kCrc32c;
  else return kCrc32;
}
template <int KIND>
constexpr uint32_t crc_poly() { return KIND == K_CRC32C ? POLY_CRC32C : POLY_CRC32; }


// acc = raw(acc, v ++ zeros(SHIFT)) with the 16 LDS tables
MC_DEV uint32_t slice16(const uint32_t *__restrict__ V, uint32_t acc, mc_u32x4 v) {
  const uint32_t d = acc ^ v.x;
  return V[0 * 256 + (d & 0xffu)] ^ V[1 * 256 + ((d >> 8) & 0xffu)] ^
         V[2 * 256 + ((d >> 16) & 0xffu)] ^ V[3 * 256 + (d >> 24)] ^
         V[4 * 256 + (v.y & 0xffu)] ^ V[5 * 256 + ((v.y >> 8) & 0xffu)] ^
         V[6 * 256 + ((v.y >> 16) & 0xffu)] ^ V[7 * 256 + (v.y >> 24)] ^
         V[8 * 256 + (v.z & 0xffu)] ^ V[9 * 256 + ((v.z >> 8) & 0xffu)] ^
         V[10 * 256 + ((v.z >> 16) & 0xffu)] ^ V[11 * 256 + (v.z >> 24)] ^
         V[12 * 256 + (v.w & 0xffu)] ^ V[13 * 256 + ((v.w >> 8) & 0xffu)] ^
         V[14 * 256 + ((v.w >> 16) & 0xffu)] ^ V[15 * 256 + (v.w >> 24)];
}

// ---------------------------------------------------------------------------
// 16-B accesses at byte position pos of a chunk of n bytes; bytes >= n read
// as 0 and are not written.  AL: 2 = 16-B aligned (nontemporal), 1 = 4-B
// aligned (global_load/store_dwordx4 at dword alignment), 0 = bytes.
// ---------------------------------------------------------------------------
template <int AL>
MC_DEV mc_u32x4 ld_vec(const uint8_t *p) {
  if constexpr (AL == 2) {
    return mc_ld16<true>(p);
  } else if constexpr (AL == 1) {
    mc_u32x4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), 16);
    return v;
  } else {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)p[4 * j] | ((uint32_t)p[4 * j + 1] << 8) | ((uint32_t)p[4 * j + 2] << 16) |
             ((uint32_t)p[4 * j + 3] << 24);
    return mc_u32x4{w[0], w[1], w[2], w[3]};
  }
}
template <int AL>
MC_DEV void st_vec(uint8_t *p, mc_u32x4 v) {
  if constexpr (AL == 2) {
    mc_st16<true>(p, v);
  } else if constexpr (AL == 1) {
    __builtin_memcpy(__builtin_assume_aligned(p, 4), &v, 16);
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 16; ++j) p[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
  }
}
template <int AL>
MC_DEV mc_u32x4 ld_masked(const uint8_t *s, size_t pos, size_t n) {
  if (pos + 16 <= n) return ld_vec<AL>(s + pos);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16; ++j)
    if (pos + j < n) w[j >> 2] |= (uint32_t)s[pos + j] << (8 * (j & 3));
  return mc_u32x4{w[0], w[1], w[2], w[3]};
}
template <int AL>
MC_DEV void st_masked(uint8_t *d, size_t pos, size_t n, mc_u32x4 v) {
  if (pos + 16 <= n) {
    st_vec<AL>(d + pos, v);
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (int j = 0; j < 16; ++j)
    if (pos + j < n) d[pos + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
}

constexpr uint32_t ADLER_P = 65521u;

MC_DEV uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
  return v;
}
MC_DEV uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

MC_DEV uint32_t load_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

MC_DEV void store_le32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

// Powers of x the CRC finalize needs, the same for every chunk of a call:
// computed once on the host (a device thread raising x to a 2^25 power with
// bit-serial products took ~7 us of serial time per call).
struct CrcFin {
  uint32_t xb[32];          // X * (bit m): basis of the product by X = x^(8 * tile bytes)
  uint32_t tail[MC_BLOCK];  // X^(tiles - hi(t)): moves thread t's fold to the chunk end
  uint32_t pad;             // x^(-8 * zero padding of the last tile)
  uint32_t xn;              // x^(8 * chunk bytes)
  uint32_t head;            // 1: the tiles started at the 4 stored bytes before the payload (aligned
                            // verify of a location="start" buffer); their share is removed at the finish
};

// tile partial words: plain, or agent-scope relaxed atomics (sc1) for the
// in-launch hand-off to the last block (MI355X_MICROARCH.md, Valid forms,
// table row 1)
template <bool SC1>
MC_DEV uint32_t ck_ld(const uint32_t *p) {
  if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// Fold chunk c's tile partials into the checksum (every thread of the
// block); write it to out[c] (if out) and/or as a little-endian footer at
// footer + c*footer_stride, and the stored footer to stored_out[c].
// (`out` / `stored_out` may be host-mapped pinned memory.)
template <int KIND, int K, bool SC1>
MC_DEV void ck_finish_chunk(const CrcFin &fin, const uint32_t *partials, size_t tiles_per_chunk, size_t n,
                            uint32_t init, uint32_t *out, uint8_t *footer, size_t footer_stride,
                            const uint8_t *stored, size_t stored_stride, uint32_t *stored_out, size_t c) {
  __shared__ uint64_t red[2][MC_BLOCK / 64];
  if (stored_out && threadIdx.x == 0) stored_out[c] = load_le32(stored + c * stored_stride);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t lo = tiles_per_chunk * threadIdx.x / MC_BLOCK;
  const size_t hi = tiles_per_chunk * (threadIdx.x + 1) / MC_BLOCK;
  uint32_t result;
  // The thread's tile partials are loaded CK_FOLD_BATCH at a time, all loads
  // issued before the first use: folded one by one, every agent-scope (sc1)
  // load waited for the previous one -- 16 serial round trips per thread, the
  // bulk of the one-launch verify's 7-9 us tail.  Indices past `hi` re-read
  // the last partial and are masked out, so the loads stay unconditional.
  constexpr int CK_FOLD_BATCH = 16;
  if constexpr (KIND == K_ADLER) {
    uint64_t s1 = 0, s2 = 0;
    for (size_t j0 = lo; j0 < hi; j0 += CK_FOLD_BATCH) {
      uint32_t a[CK_FOLD_BATCH], b[CK_FOLD_BATCH];
#pragma unroll
      for (int u = 0; u < CK_FOLD_BATCH; ++u) {
        const size_t j = j0 + u < hi ? j0 + u : hi - 1;
        a[u] = ck_ld<SC1>(&partials[2 * (c * tiles_per_chunk + j)]);
        b[u] = ck_ld<SC1>(&partials[2 * (c * tiles_per_chunk + j) + 1]);
      }
#pragma unroll
      for (int u = 0; u < CK_FOLD_BATCH; ++u)
        if (j0 + u < hi) {
          s1 += a[u];
          s2 += b[u];
        }
    }
    s1 = wave_sum(s1 % ADLER_P);
    s2 = wave_sum(s2 % ADLER_P);
    if (lane == 0) {
      red[0][wave] = s1;
      red[1][wave] = s2;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint64_t x = 0, y = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) {
      x += red[0][w];
      y += red[1][w];
    }
    // zlib.adler32(data, value): a0 = value & 0xffff, b0 = value >> 16
    const uint64_t a0 = init & 0xffffu, b0 = init >> 16;
    const uint64_t a = (a0 + x) % ADLER_P;
    const uint64_t b = (b0 + (n % ADLER_P) * a0 + y) % ADLER_P;
    result = (uint32_t)((b << 16) | a);
  } else {
    // Horner over this thread's tiles; the product by the constant X is
    // linear in the bits of acc: 4 byte tables in LDS built from X's basis
    __shared__ uint32_t T[4][256];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t r = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if ((threadIdx.x >> k) & 1) r ^= fin.xb[8 * j + k];
      T[j][threadIdx.x] = r;
    }
    __syncthreads();
    uint32_t acc = 0;
    if constexpr (SC1) {  // the one-launch finish: agent-scope loads, batched
      for (size_t j0 = lo; j0 < hi; j0 += CK_FOLD_BATCH) {
        uint32_t v[CK_FOLD_BATCH];
#pragma unroll
        for (int u = 0; u < CK_FOLD_BATCH; ++u)
          v[u] = ck_ld<SC1>(&partials[c * tiles_per_chunk + (j0 + u < hi ? j0 + u : hi - 1)]);
#pragma unroll
        for (int u = 0; u < CK_FOLD_BATCH; ++u)
          if (j0 + u < hi)
            acc = (T[0][acc & 0xffu] ^ T[1][(acc >> 8) & 0xffu] ^ T[2][(acc >> 16) & 0xffu] ^ T[3][acc >> 24]) ^
                  v[u];
      }
    } else {  // the finalize kernel: plain loads pipeline by themselves (batching measured 7.2 -> 10.5 us)
#pragma unroll 4
      for (size_t j = lo; j < hi; ++j)
        acc = (T[0][acc & 0xffu] ^ T[1][(acc >> 8) & 0xffu] ^ T[2][(acc >> 16) & 0xffu] ^ T[3][acc >> 24]) ^
              partials[c * tiles_per_chunk + j];
    }
    if (hi > lo) acc = gf_mul(acc, fin.tail[threadIdx.x], crc_poly<KIND>());
    acc = wave_xor(acc);
    if (lane == 0) red[0][wave] = acc;
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint32_t r = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) r ^= (uint32_t)red[0][w];
    // r covers tiles_per_chunk * TB bytes; the last (TB*tiles - n) are padding
    r = gf_mul(r, fin.pad, crc_poly<KIND>());
    if (fin.head) {  // raw(0, payload) = raw(0, stored4 ++ payload) ^ raw(0, stored4) * x^(8n)
      uint32_t hw = load_le32(stored + c * stored_stride);
#pragma unroll
      for (int i = 0; i < 32; ++i) hw = (hw >> 1) ^ ((hw & 1u) ? crc_poly<KIND>() : 0u);
      r ^= gf_mul(hw, fin.xn, crc_poly<KIND>());
    }
    // crc(D, value) = ~raw(~value, D) = ~(~value * x^(8n) xor raw(0, D))
    result = ~(gf_mul(~init, fin.xn, crc_poly<KIND>()) ^ r);
  }
  if (out) out[c] = result;
  if (footer) store_le32(footer + c * footer_stride, result);
}


// ---------------------------------------------------------------------------
// Per-tile partials.  Block loops over tiles (tile = chunk * tiles_per_chunk
// + t); the CRC tables are staged into LDS once per block.
//   CRC:   partials[tile] = raw(0, tile bytes ++ zero padding to K*STEP)
//   Adler: partials[2*tile] = S1 mod P, partials[2*tile+1] = S2 mod P
// COPY: also write the payload to dst (+ per-row offset already applied).
// ---------------------------------------------------------------------------
// FUSED (one chunk): partials are stored sc1 and every block arrives
// (mc_arrive_last, sharded counter) after a vmcnt(0) wait; the last block
// folds them in the same launch (ck_finish_chunk) and zeroes the counter
// again -- one launch, no finalize boundary.
struct CkFinish {
  uint32_t init, seq;  // seq: published after the verdict (mc_publish_verdict_seq)
  uint32_t head;       // 4: the tiles cover the 4 stored bytes before the payload (see CrcFin::head)
  uint32_t *ticket, *out, *stored_out;
  uint8_t *footer;
  size_t footer_stride;
  const uint8_t *stored;
};

// Adler32's one-launch finish needs no partial stores at all: a block's
// tiles add up (absolute weights), and its (S1, S2) mod P travel inside ONE
// returning 64-bit atomic on its shard's word, packed as count (bits 0-7),
// sum of S1 (8-31), sum of S2 (32-55) -- at most 255 blocks per shard keep
// every field from carrying into the next.  The shard's last arriver holds
// the shard's sums and adds them (mod P) into the top word the same way; the
// top's last arriver finishes the chunk.  Each last arriver zeroes the word
// it closed, so the ticket is left zero.  No vmcnt wait for hand-off stores,
// no fold over per-tile partials.
constexpr unsigned ADLER_MAX_GRID = MC_ARRIVAL_SHARDS * 255u;


// FUSED (one chunk) CRC finish: every block arrives after its sc1 partial
// stores drained; the last one folds the partials and publishes the verdict.
template <int KIND, int K>
MC_DEV void ck_fused_tail(const CrcFin &fin, const uint32_t *partials, size_t tiles_per_chunk, size_t n,
                          size_t src_stride, const CkFinish &fx) {
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {  // every block has at least one tile (grid <= tiles)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = mc_arrive_last(fx.ticket, gridDim.x);
  }
  __syncthreads();
  if (!last) return;
  ck_finish_chunk<KIND, K, true>(fin, partials, tiles_per_chunk, n, fx.init, fx.out, fx.footer,
                                 fx.footer_stride, fx.stored, src_stride, fx.stored_out, 0);
  if (threadIdx.x == 0) {  // thread 0 wrote both verdict words
    mc_publish_verdict_seq(fx.out, fx.seq);
    mc_arrivals_reset(fx.ticket);  // left zero for the next launch
  }
}

template <int KIND>
MC_DEV uint32_t mulx_r(uint32_t a) {  // a * x mod P (reflected)
  return (a >> 1) ^ ((uint32_t)__builtin_amdgcn_sbfe((int)a, 0, 1) & crc_poly<KIND>());
}


// bit-sliced CRC tiles (mc_crc_bs.hip): the kernel for tiles of K >= 4
// vectors per lane; kind MC_CK_CRC32 / MC_CK_CRC32C, als / ald = align class
// of source / destination (2: 16 B, 1: 4 B, 0: bytes), dst NULL = no copy,
// fx NULL = partials only (separate finalize).  Returns MC_EINVAL for an
// unsupported combination.
int launch_crc_bs(int kind, int K, int als, int ald, const uint8_t *s, size_t ss, uint8_t *d, size_t ds,
                  size_t n, size_t tpc, size_t total, uint32_t *parts, const CrcFin &fin, const CkFinish *fx,
                  unsigned grid, hipStream_t st);

}  // namespace mcck
