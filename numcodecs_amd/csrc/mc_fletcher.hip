// mc_fletcher.hip -- Fletcher32 (fletcher32.pyx:24-115) for gfx950, alone and
// fused with Shuffle over batches of chunks.
//
// The reference loop (HDF5 H5checksum.c) adds big-endian 16-bit words,
// sum1 += w; sum2 += sum1, folding both sums every 360 words with
// x = (x & 0xffff) + (x >> 16) and twice at the end.  Folding preserves the
// value mod 65535 and never turns a positive sum into 0, and the 360-word
// blocks keep the uint32 sums from overflowing, so with n = ceil(len/2) words
// (an odd trailing byte is the high byte of a last word):
//     S1 = sum_i w_i,   S2 = sum_i (n - i) * w_i
//     result = (r(S2) << 16) | r(S1),  r(S) = 0 if S == 0 else ((S-1) mod 65535) + 1
// and S == 0 exactly when every word is zero.  With absolute weights (n - i)
// any partition of the words into slices adds up mod 65535, which makes the
// checksum a plain parallel reduction: lanes accumulate 16-B vectors (8 words)
// as S1 += A, S2 += c*A - B with A = sum w_m, B = sum m*w_m, c = (n - j0) mod
// 65535; workgroups reduce through wave shuffles and LDS; partials per
// (chunk, slice) are folded by a small finalize kernel that also writes the
// little-endian footer (_utils.pxd:11-24) or compares against it.
#include "mc_shuffle.h"

namespace {

constexpr uint32_t M = 65535u;

struct F32Part {
  uint64_t s1;   // sum of words
  uint64_t s2a;  // sum of c * A
  uint64_t s2b;  // sum of B (intra-vector weights)
  uint32_t nz;   // OR of all words
};

MC_DEV void part_init(F32Part &p) { p.s1 = p.s2a = p.s2b = 0; p.nz = 0; }

// the two big-endian words of a little-endian dword: w0 = bytes(0,1), w1 = bytes(2,3)
MC_DEV uint32_t be_swap16x2(uint32_t x) { return mc_perm(0u, x, 0x02030001u); }

// one word with weight c
MC_DEV void part_word(F32Part &p, uint32_t w, uint32_t c) {
  p.s1 += w;
  p.s2a += (uint64_t)c * w;
  p.nz |= w;
}

MC_DEV uint32_t mod_m(uint64_t x) { return (uint32_t)(x % M); }

// A run of up to RUN_MAX consecutive 16-B vectors of one thread whose k-th
// vector's first word has weight c0 - k*step (mod M).  Per vector only the
// word sum A (a v_dot2_u32_u16 chain into the running prefix P) and the
// intra-vector weighted sum B (a second chain) are accumulated, plus U += P;
// the weights are applied once per run:
//   sum_k c_k*A_k - B = c0*P - step*sum_k k*A_k - B,  sum_k k*A_k = k*P - U
// (mod M).  13 VALU ops per vector against ~35 for unpacking the 8 words
// and weighting each vector separately.
constexpr uint32_t RUN_MAX = 64;  // keeps U < 2^31, B < 2^27
typedef unsigned short f32_u16x2 __attribute__((ext_vector_type(2)));
MC_DEV uint32_t dot2u(uint32_t a, uint32_t w, uint32_t c) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(f32_u16x2, a), __builtin_bit_cast(f32_u16x2, w), c, false);
}
struct F32Run {
  uint32_t P, U, B, k, c0;
};
MC_DEV void run_start(F32Run &r, uint32_t c0) {
  r.P = r.U = r.B = r.k = 0;
  r.c0 = c0;
}
MC_DEV void run_vec(F32Run &r, mc_u32x4 v) {
  const uint32_t y0 = be_swap16x2(v.x), y1 = be_swap16x2(v.y);
  const uint32_t y2 = be_swap16x2(v.z), y3 = be_swap16x2(v.w);
  uint32_t P = dot2u(y0, 0x00010001u, r.P);
  P = dot2u(y1, 0x00010001u, P);
  P = dot2u(y2, 0x00010001u, P);
  P = dot2u(y3, 0x00010001u, P);
  uint32_t B = dot2u(y0, 0x00010000u, r.B);  // words 0..7 weighted 0..7
  B = dot2u(y1, 0x00030002u, B);
  B = dot2u(y2, 0x00050004u, B);
  B = dot2u(y3, 0x00070006u, B);
  r.P = P;
  r.U += P;
  r.B = B;
  ++r.k;
}
// fold the run into p (S1 exact, S2 mod M, nz) and start the next run at
// weight c0 - k*step
MC_DEV void run_fold(F32Part &p, F32Run &r, uint32_t step) {
  if (!r.k) return;
  const uint64_t P = r.P;
  const uint64_t T2 = (uint64_t)r.k * P - r.U;  // sum_k k*A_k, exact
  const uint32_t a = (uint32_t)(((uint64_t)r.c0 * (P % M)) % M);
  const uint32_t t = (uint32_t)(((uint64_t)step * (T2 % M)) % M);
  const uint32_t b = r.B % M;
  p.s1 += P;
  p.s2a += (a + 2 * M - t - b) % M;
  p.nz |= (uint32_t)(P != 0);  // a word sum is 0 only if every word is
  const uint32_t adv = (uint32_t)(((uint64_t)r.k * step) % M);
  run_start(r, r.c0 >= adv ? r.c0 - adv : r.c0 + M - adv);
}

// reduce a thread's partial to {S1 mod M, S2 mod M, nz} across the block;
// valid in thread 0.
MC_DEV void block_reduce(const F32Part &p, uint32_t &s1, uint32_t &s2, uint32_t &nz) {
  __shared__ uint32_t red[3][MC_BLOCK / 64];
  uint64_t a = mod_m(p.s1);
  uint64_t b = (mod_m(p.s2a) + M - mod_m(p.s2b)) % M;
  uint32_t z = p.nz;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_down(a, off, 64);
    b += __shfl_down(b, off, 64);
    z |= __shfl_down(z, off, 64);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = mod_m(a);
    red[1][wave] = mod_m(b);
    red[2][wave] = z;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t x = 0, y = 0;
    uint32_t q = 0;
    for (int w = 0; w < MC_BLOCK / 64; ++w) {
      x += red[0][w];
      y += red[1][w];
      q |= red[2][w];
    }
    s1 = mod_m(x);
    s2 = mod_m(y);
    nz = q;
  }
}

MC_DEV uint32_t final_sum(uint32_t s1, uint32_t s2, uint32_t nz) {
  if (!nz) return 0u;
  const uint32_t r1 = (s1 + M - 1) % M + 1, r2 = (s2 + M - 1) % M + 1;
  return (r2 << 16) | r1;
}

MC_DEV void store_le32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
MC_DEV uint32_t load_le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// 16-B vector access; AL = 2: 16-B aligned (nontemporal), 1: 4-B aligned
// (global_load/store_dwordx4 at dword alignment: rows of chunk_bytes + 4)
template <int AL, bool NT = true>
MC_DEV mc_u32x4 f32_ld(const uint8_t *p) {
  if constexpr (AL == 2) {
    return mc_ld16<NT>(p);
  } else {
    mc_u32x4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 4), 16);
    return v;
  }
}
template <int AL>
MC_DEV void f32_st(uint8_t *p, mc_u32x4 v) {
  if constexpr (AL == 2) mc_st16<true>(p, v);
  else __builtin_memcpy(__builtin_assume_aligned(p, 4), &v, 16);
}

// ---------------------------------------------------------------------------
// checksum (optionally fused with a copy) over slices of chunks
// block = (chunk c, slice sl); partials[block] = {S1, S2, nz}
// AL: alignment class of src/dst rows (above); 0 = bytes only
// ---------------------------------------------------------------------------
enum FinalMode { F_SUM = 0, F_FOOTER = 1, F_VERIFY = 2 };

// partial words of a (chunk, slice) block: plain, or agent-scope relaxed
// atomics (global_load/store ... sc1) for the in-launch hand-off to the last
// block of a chunk (MI355X_MICROARCH.md, Valid forms, table row 1: one lane
// per storing workgroup stores sc1, waits vmcnt(0), adds to ONE counter; the
// workgroup whose add came last loads sc1 after a barrier)
template <bool SC1>
MC_DEV uint32_t part_ld(const uint32_t *p) {
  if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// Fold chunk c's slice partials and finish it (every thread of the block):
//   F_SUM:    out[c] = checksum
//   F_FOOTER: LE32 checksum at dst + c*dst_stride + nbytes (and out[c] if set)
//   F_VERIFY: out[2c] = checksum, out[2c+1] = LE32 footer at src + c*src_stride + nbytes
// (`out` may be host-mapped pinned memory: the public decode reads its
// verdict from there after one stream sync)
template <bool SC1>
MC_DEV void f32_finish_chunk(const uint32_t *partials, unsigned nslices, size_t c, int mode,
                             const uint8_t *src, size_t src_stride, uint8_t *dst, size_t dst_stride,
                             size_t nbytes, uint32_t *out, uint32_t seq = 0);

// one-launch finish (k_f32_partial with `tickets`): the packed arrival word
// {count, S1 sum, S2 sum, nonzero count}; at most 255 blocks per shard
constexpr unsigned F32_MAX_FUSED_GRID = MC_ARRIVAL_SHARDS * 255u;
MC_DEV unsigned long long f32_pack(uint32_t s1, uint32_t s2, bool nz) {
  return ((unsigned long long)nz << 56) | ((unsigned long long)s2 << 32) | ((unsigned long long)s1 << 8) | 1ull;
}

// chunk c's checksum f to where `mode` puts it (F_SUM: out[c]; F_FOOTER: LE32
// footer after the payload in dst, and out[c] if set; F_VERIFY: out[2c] = f,
// out[2c+1] = the stored footer, then `seq` published)
MC_DEV void f32_write_result(uint32_t f, size_t c, int mode, const uint8_t *src, size_t src_stride, uint8_t *dst,
                             size_t dst_stride, size_t nbytes, uint32_t *out, uint32_t seq) {
  if (mode == F_SUM) {
    out[c] = f;
  } else if (mode == F_FOOTER) {
    store_le32(dst + c * dst_stride + nbytes, f);
    if (out) out[c] = f;
  } else {
    out[2 * c] = f;
    out[2 * c + 1] = load_le32(src + c * src_stride + nbytes);
    mc_publish_verdict_seq(out, seq);
  }
}

// block = (chunk c, slice sl), partials[block] = {S1, S2, nz}; or, with
// `tickets` (one chunk, FUSED finish): block b sums slices b, b + grid, ...
// (absolute weights: slice partials add; the launch gives one slice per
// block), stores ONE partial sc1 and arrives; the fold runs in this launch
// (below).  `seq` != 0: F_VERIFY publishes out[2] = seq after the verdict
template <bool COPY, int AL, int F32_UNROLL, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_f32_partial(
    const uint8_t *__restrict__ src, size_t src_stride, uint8_t *__restrict__ dst,
    size_t dst_stride, size_t nbytes, unsigned nslices, uint32_t *__restrict__ partials,
    uint32_t *tickets, int mode, uint32_t *out, uint32_t seq) {
  const size_t c = tickets ? 0 : blockIdx.x / nslices;
  const unsigned sl0 = tickets ? blockIdx.x : blockIdx.x - (unsigned)(c * nslices);
  const unsigned sl_step = tickets ? gridDim.x : nslices;
  const uint8_t *s = src + c * src_stride;
  uint8_t *d = COPY ? dst + c * dst_stride : nullptr;
  const uint64_t nwords = (nbytes + 1) / 2;
  const size_t nvec = AL ? nbytes / 16 : 0;
  F32Part p;
  part_init(p);
  for (unsigned sl = sl0; sl < nslices; sl += sl_step) {
    const size_t v_lo = nvec * sl / nslices, v_hi = nvec * (sl + 1) / nslices;
    size_t v = v_lo + threadIdx.x;
    // weight of the vector's first word, stepped by 8*MC_BLOCK words per iteration
    uint32_t cw = (uint32_t)((nwords - 8 * (uint64_t)v) % M);
    constexpr uint32_t STEP = (8u * MC_BLOCK) % M;
    F32Run r;
    run_start(r, cw);
    // F32_UNROLL vectors in flight per thread before any is consumed
    for (; v + (F32_UNROLL - 1) * MC_BLOCK < v_hi; v += F32_UNROLL * MC_BLOCK) {
      mc_u32x4 x[F32_UNROLL];
#pragma unroll
      for (int j = 0; j < F32_UNROLL; ++j) x[j] = f32_ld<AL, NT>(s + (v + j * MC_BLOCK) * 16);
#pragma unroll
      for (int j = 0; j < F32_UNROLL; ++j) {
        if constexpr (COPY) f32_st<AL>(d + (v + j * MC_BLOCK) * 16, x[j]);
        run_vec(r, x[j]);
      }
      if (r.k > RUN_MAX - F32_UNROLL) run_fold(p, r, STEP);
    }
    for (; v < v_hi; v += MC_BLOCK) {
      const mc_u32x4 x = f32_ld<AL>(s + v * 16);
      if constexpr (COPY) f32_st<AL>(d + v * 16, x);
      run_vec(r, x);
    }
    run_fold(p, r, STEP);
    if (sl == nslices - 1) {  // bytes after the last whole vector, word by word
      const size_t b0 = nvec * 16;
      for (size_t b = b0 + 2 * (size_t)threadIdx.x; b < nbytes; b += 2 * MC_BLOCK) {
        const uint32_t hi = s[b];
        const uint32_t lo = b + 1 < nbytes ? s[b + 1] : 0u;
        if constexpr (COPY) {
          d[b] = (uint8_t)hi;
          if (b + 1 < nbytes) d[b + 1] = (uint8_t)lo;
        }
        part_word(p, (hi << 8) | lo, (uint32_t)((nwords - b / 2) % M));
      }
    }
  }
  uint32_t s1, s2, nz;
  block_reduce(p, s1, s2, nz);
  if (!tickets) {  // a separate finalize launch folds the partials
    if (threadIdx.x == 0) {
      partials[3 * (size_t)blockIdx.x + 0] = s1;
      partials[3 * (size_t)blockIdx.x + 1] = s2;
      partials[3 * (size_t)blockIdx.x + 2] = nz;
    }
    return;
  }
  // fused finish in this launch (no finalize kernel, no partial stores): the
  // block's {S1 mod M, S2 mod M, nz} travel inside ONE returning 64-bit
  // atomic on its shard's word (block b in shard b % 64), packed as count
  // (bits 0-7), sum of S1 (8-31), sum of S2 (32-55), count of nonzero blocks
  // (56-63) -- at most F32_MAX_FUSED_GRID blocks keep every field from
  // carrying.  The shard's last arriver holds the shard's sums and adds them
  // into the top word the same way; the top's last arriver finishes the
  // chunk.  Each last arriver zeroes the word it closed (left zero).  (The
  // previous form stored partials sc1, waited for the stores, arrived, and
  // had the last blocks fold them: ~3 us more per verify.)
  if (threadIdx.x != 0) return;
  const unsigned sh = mc_arrival_shard(blockIdx.x);
  unsigned long long *w = reinterpret_cast<unsigned long long *>(tickets + MC_ARRIVAL_LINE * sh);
  const unsigned long long old = atomicAdd(w, f32_pack(s1, s2, nz != 0));
  if ((old & 0xffu) + 1u != mc_arrival_per(sh, gridDim.x)) return;
  *w = 0;  // every arrival of this shard is in
  const uint32_t t1 = mod_m(((old >> 8) & 0xffffffu) + s1), t2 = mod_m(((old >> 32) & 0xffffffu) + s2);
  const bool tz = (old >> 56) != 0 || nz != 0;
  unsigned long long *t = reinterpret_cast<unsigned long long *>(tickets + MC_ARRIVAL_LINE * MC_ARRIVAL_SHARDS);
  const unsigned long long top = atomicAdd(t, f32_pack(t1, t2, tz));
  if ((top & 0xffu) + 1u != mc_arrival_nshards(gridDim.x)) return;
  *t = 0;
  const uint32_t a = mod_m(((top >> 8) & 0xffffffu) + t1), b = mod_m(((top >> 32) & 0xffffffu) + t2);
  const bool z = (top >> 56) != 0 || tz;
  f32_write_result(final_sum(a, b, z ? 1u : 0u), 0, mode, src, src_stride, dst, dst_stride, nbytes, out, seq);
}

template <bool SC1>
MC_DEV void f32_finish_chunk(const uint32_t *partials, unsigned nslices, size_t c, int mode,
                             const uint8_t *src, size_t src_stride, uint8_t *dst, size_t dst_stride,
                             size_t nbytes, uint32_t *out, uint32_t seq) {
  F32Part p;
  part_init(p);
#pragma unroll 8
  for (unsigned sl = threadIdx.x; sl < nslices; sl += MC_BLOCK) {
    const uint32_t *q = partials + 3 * (c * nslices + sl);
    p.s1 += part_ld<SC1>(q);
    p.s2a += part_ld<SC1>(q + 1);  // partial S2 already reduced: s2b stays 0
    p.nz |= part_ld<SC1>(q + 2);
  }
  uint32_t a, b, z;
  block_reduce(p, a, b, z);
  if (threadIdx.x != 0) return;
  f32_write_result(final_sum(a, b, z), c, mode, src, src_stride, dst, dst_stride, nbytes, out, seq);
}

// one workgroup per chunk: the 256 threads fold the chunk's slices (a large
// chunk has thousands: a single thread walking them serially was the
// bottleneck of a 256 MiB checksum) -- f32_finish_chunk
__global__ __launch_bounds__(MC_BLOCK) void k_f32_finalize(
    const uint32_t *__restrict__ partials, unsigned nslices, size_t nchunks, int mode,
    const uint8_t *__restrict__ src, size_t src_stride, uint8_t *__restrict__ dst,
    size_t dst_stride, size_t nbytes, uint32_t *__restrict__ out) {
  (void)nchunks;
  f32_finish_chunk<false>(partials, nslices, blockIdx.x, mode, src, src_stride, dst, dst_stride, nbytes, out);
}

// ---------------------------------------------------------------------------
// fused Shuffle(es) + Fletcher32 over batches of chunks, one tile per block
// (register layout of mc_shuffle.hip).  Needs count % TE == 0.
// ---------------------------------------------------------------------------
// Per-thread accumulation over the plane dwords of a tile: the dword at plane
// byte offset b*count + e (e even, quad q) is word j = (b*count + e)/2, with
// weight c(q, b) = (nwords - j) mod M = cb0 - b*cnt_m - 2*MC_BLOCK*q (mod M)
// (cb0 = (nwords - e0/2) mod M, cnt_m = (count/2) mod M), so sum c*A = cb0*SA - cnt_m*SbA - 2*MC_BLOCK*SqA (mod M)
// with SA = sum A, SbA = sum b*A, SqA = sum q*A: four v_dot2_u32_u16 per
// dword (b and q are compile-time constants) instead of a modulo and an
// unpacking per dword.  Bounds: Q*ES <= 64 dwords per thread keeps every
// sum below 2^29.
struct PlaneSums {
  uint32_t SA, SbA, SqA, SB;
};
MC_DEV void plane_init(PlaneSums &t) { t.SA = t.SbA = t.SqA = t.SB = 0; }
MC_DEV void plane_dword(PlaneSums &t, uint32_t x, uint32_t b, uint32_t q) {
  const uint32_t y = be_swap16x2(x);  // w0 in the low half, w1 in the high half
  t.SA = dot2u(y, 0x00010001u, t.SA);
  t.SbA = dot2u(y, b * 0x00010001u, t.SbA);
  t.SqA = dot2u(y, q * 0x00010001u, t.SqA);
  t.SB = dot2u(y, 0x00010000u, t.SB);  // the dword's second word: weight offset 1
}
MC_DEV void plane_fold(F32Part &p, const PlaneSums &t, uint32_t cb0, uint32_t cnt_m) {
  constexpr uint32_t QW = (2u * MC_BLOCK) % M;
  const uint64_t a = (uint64_t)cb0 * (t.SA % M) + (uint64_t)(M - cnt_m) * (t.SbA % M) +
                     (uint64_t)(M - QW) * (t.SqA % M);
  p.s1 += t.SA;
  p.s2a += a % M;
  p.s2b += t.SB;
  p.nz |= (uint32_t)(t.SA != 0);
}

template <int ES, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_shuffle_f32_enc(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    uint32_t *__restrict__ partials) {
  using G = Geom<ES, 1>;
  const int tid = threadIdx.x;
  const size_t tile = blockIdx.x;
  const size_t c = tile / m.tiles_per_chunk;
  const size_t t = tile - c * m.tiles_per_chunk;
  const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TB;
  uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TE;
  const uint64_t nwords = (uint64_t)m.count * ES / 2;
  const size_t e0 = t * (size_t)G::TE + 4 * (size_t)tid;
  const uint32_t cb0 = (uint32_t)((nwords - e0 / 2) % M);
  const uint32_t cnt_m = (uint32_t)((m.count / 2) % M);
  uint32_t w[G::Q][ES];
#pragma unroll
  for (int q = 0; q < G::Q; ++q) load_quad<ES, NT>(s + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w[q]);
  static_assert(G::Q * ES <= 64, "PlaneSums bounds");
  PlaneSums ps;
  plane_init(ps);
#pragma unroll
  for (int q = 0; q < G::Q; ++q) {
    uint32_t pl[ES];
    mc_quad_to_planes<ES>(w[q], pl);
#pragma unroll
    for (int b = 0; b < ES; ++b) {
      mc_st4<NT>(d + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4, pl[b]);
      plane_dword(ps, pl[b], b, q);
    }
  }
  F32Part p;
  part_init(p);
  plane_fold(p, ps, cb0, cnt_m);
  uint32_t s1, s2, nz;
  block_reduce(p, s1, s2, nz);
  if (tid == 0) {
    partials[3 * tile + 0] = s1;
    partials[3 * tile + 1] = s2;
    partials[3 * tile + 2] = nz;
  }
}

template <int ES, bool NT>
__global__ __launch_bounds__(MC_BLOCK) void k_f32_unshuffle(
    const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, ChunkMap m,
    uint32_t *__restrict__ partials) {
  using G = Geom<ES, 1>;
  const int tid = threadIdx.x;
  const size_t tile = blockIdx.x;
  const size_t c = tile / m.tiles_per_chunk;
  const size_t t = tile - c * m.tiles_per_chunk;
  const uint8_t *s = src + c * m.src_stride + t * (size_t)G::TE;
  uint8_t *d = dst + c * m.dst_stride + t * (size_t)G::TB;
  const uint64_t nwords = (uint64_t)m.count * ES / 2;
  const size_t e0 = t * (size_t)G::TE + 4 * (size_t)tid;
  const uint32_t cb0 = (uint32_t)((nwords - e0 / 2) % M);
  const uint32_t cnt_m = (uint32_t)((m.count / 2) % M);
  uint32_t p[G::Q][ES];
#pragma unroll
  for (int b = 0; b < ES; ++b)
#pragma unroll
    for (int q = 0; q < G::Q; ++q)
      p[q][b] = mc_ld4<NT>(s + (size_t)b * m.count + (size_t)(q * MC_BLOCK + tid) * 4);
  static_assert(G::Q * ES <= 64, "PlaneSums bounds");
  PlaneSums ps;
  plane_init(ps);
#pragma unroll
  for (int q = 0; q < G::Q; ++q) {
#pragma unroll
    for (int b = 0; b < ES; ++b) plane_dword(ps, p[q][b], b, q);
    uint32_t w[ES];
    mc_planes_to_quad<ES>(p[q], w);
    store_quad<ES, NT>(d + (size_t)(q * MC_BLOCK + tid) * 4 * ES, w);
  }
  F32Part acc;
  part_init(acc);
  plane_fold(acc, ps, cb0, cnt_m);
  uint32_t s1, s2, nz;
  block_reduce(acc, s1, s2, nz);
  if (tid == 0) {
    partials[3 * tile + 0] = s1;
    partials[3 * tile + 1] = s2;
    partials[3 * tile + 2] = nz;
  }
}

// slices per chunk for the standalone checksum: ~32 KiB of payload per block,
// at least one block per chunk
static size_t f32_slice_bytes();

static unsigned slices_for(size_t nbytes, size_t nchunks) {
  size_t sl = nbytes / f32_slice_bytes();
  if (sl < 1) sl = 1;
  if (sl > 65536) sl = 65536;
  // keep the grid within a 32-bit block count
  while (sl > 1 && sl * nchunks > 0x7fffffffull) sl >>= 1;
  (void)nchunks;
  return (unsigned)sl;
}

static size_t partials_bytes(size_t nchunks, unsigned nslices) {
  return nchunks * (size_t)nslices * 3 * sizeof(uint32_t);
}
// the fused verify's shard-major partials (64 shards of ceil(nslices / 64))
// plus the 64 shard sums
static size_t fused_partials_bytes(unsigned nslices) {
  const size_t per_max = ((size_t)nslices + MC_ARRIVAL_SHARDS - 1) / MC_ARRIVAL_SHARDS;
  return (per_max + 1) * MC_ARRIVAL_SHARDS * 3 * sizeof(uint32_t);
}

// schedule (mc_sched.h): f32_unroll = vectors in flight per thread in
// k_f32_partial (1, 4, 8); f32_ntld = nontemporal loads (0/1); f32_slice_kb
// = payload KiB per workgroup.  Defaults from the sweep on 64 x 4 MiB rows
// (profiles/r01/fletcher32_knobs_ab.jsonl): 4 loads in flight and 32 KiB
// slices take the one-pass decode from 116 to 100 us.
// The one-launch single-chunk verify (no copy) defaults to 8 vectors in
// flight (256 MiB verify kernel 44.1-44.3 us at (grid 2048, 4 vectors) ->
// 43.0 us at (4096, 8), interleaved A/B on MI355X; the copying and batched
// passes keep 4; profiles/r01/fletcher32_knobs_ab.jsonl) and, since round 6,
// a 2048-block grid: with 8 vectors, 32 KiB slices, 43.7 / 46.4 us back to
// back / single against 44.0 / 47.6 at 4096 (tools/probe_f32_verify_sched.py,
// profiles/r06/probe_f32_verify_sched.jsonl).
static int f32_unroll(bool fused_verify = false) {
  const int e = mc_sched.f32_unroll;
  if (e == 1 || e == 4 || e == 8) return e;
  return fused_verify ? 8 : 4;
}
static bool f32_ntld() { return mc_sched.f32_ntld != 0; }
// f32_fused_grid: block cap of the one-launch verify (256 .. 65536)
static unsigned f32_fused_grid() {
  const int e = mc_sched.f32_fused_grid;
  return (unsigned)(e >= 256 && e <= 65536 ? e : 2048);
}
static size_t f32_slice_bytes() {
  const int e = mc_sched.f32_slice_kb;
  return (size_t)(e >= 4 && e <= 4096 ? e : 32) * 1024;
}

static int align_class(const void *p, size_t stride, size_t nchunks) {
  const uintptr_t a = (uintptr_t)p | (nchunks > 1 ? stride : 0);
  return a % 16 == 0 ? 2 : a % 4 == 0 ? 1 : 0;
}

static void launch_partial(const uint8_t *src, size_t src_stride, uint8_t *dst, size_t dst_stride,
                           size_t nchunks, size_t nbytes, unsigned nsl, uint32_t *partials,
                           uint32_t *tickets, int mode, uint32_t *out, uint32_t seq, hipStream_t st) {
  int al = align_class(src, src_stride, nchunks);
  if (dst) {
    const int ad = align_class(dst, dst_stride, nchunks);
    al = al < ad ? al : ad;
  }
  // fused (one chunk): at most f32_fused_grid() blocks, each summing
  // nsl / grid slices (loads only, so a looping block keeps its loads in
  // flight); the packed arrival (64 shards) keeps the tail short
  const unsigned fg = f32_fused_grid();
  const int unroll = f32_unroll(tickets && !dst);
  // (the fused encode keeps one slice per block, as the two-launch copy does)
  unsigned grid = tickets && !dst ? (nsl < fg ? nsl : fg) : (unsigned)(nchunks * nsl);
  if (tickets && grid > F32_MAX_FUSED_GRID) grid = F32_MAX_FUSED_GRID;  // packed arrival fields
#define MC_F32_U(CP, AL, U)                                                                   \
  do {                                                                                         \
    if (f32_ntld())                                                                            \
      k_f32_partial<CP, AL, U, true><<<grid, MC_BLOCK, 0, st>>>(src, src_stride, dst,          \
                                                                dst_stride, nbytes, nsl,       \
                                                                partials, tickets, mode, out, seq); \
    else                                                                                       \
      k_f32_partial<CP, AL, U, false><<<grid, MC_BLOCK, 0, st>>>(src, src_stride, dst,         \
                                                                 dst_stride, nbytes, nsl,      \
                                                                 partials, tickets, mode, out, seq);\
  } while (0)
#define MC_F32_LAUNCH(CP, AL)                                                                 \
  do {                                                                                         \
    if (unroll == 8) MC_F32_U(CP, AL, 8);                                                          \
    else if (unroll == 4) MC_F32_U(CP, AL, 4);                                                     \
    else MC_F32_U(CP, AL, 1);                                                                  \
  } while (0)
  if (dst) {
    if (al == 2) MC_F32_LAUNCH(true, 2);
    else if (al == 1) MC_F32_LAUNCH(true, 1);
    else MC_F32_LAUNCH(true, 0);
  } else {
    if (al == 2) MC_F32_LAUNCH(false, 2);
    else if (al == 1) MC_F32_LAUNCH(false, 1);
    else MC_F32_LAUNCH(false, 0);
  }
#undef MC_F32_LAUNCH
#undef MC_F32_U
}

// standalone driver: checksum (+ optional copy) of nchunks chunks, then
// finalize -- in the same launch when `tickets` (MC_ARRIVAL_WORDS zeroed
// words, left zeroed; one chunk only) is given, else as a second launch
static int f32_run(const uint8_t *src, size_t src_stride, uint8_t *dst, size_t dst_stride,
                   size_t nchunks, size_t nbytes, int mode, uint32_t *out, void *ws,
                   size_t ws_bytes, hipStream_t st, uint32_t *tickets = nullptr, uint32_t seq = 0) {
  const unsigned nsl = slices_for(nbytes, nchunks);
  const size_t need = tickets ? fused_partials_bytes(nsl) : partials_bytes(nchunks, nsl);
  if (!ws || ws_bytes < need) return MC_ENOSPC;
  uint32_t *partials = static_cast<uint32_t *>(ws);
  // F_FOOTER copies the payload in front of its footer; F_VERIFY with a dst
  // compacts the payloads out of the encoded rows (the decode pass)
  const bool copy = dst != nullptr;
  launch_partial(src, src_stride, copy ? dst : nullptr, dst_stride, nchunks, nbytes, nsl, partials, tickets, mode,
                 out, seq, st);
  int rc = mc_last_launch();
  if (rc != MC_OK || tickets) return rc;
  k_f32_finalize<<<(unsigned)nchunks, MC_BLOCK, 0, st>>>(partials, nsl, nchunks, mode, src, src_stride,
                                                         dst, dst_stride, nbytes, out);
  return mc_last_launch();
}

static size_t fused_tile_elems(size_t es) { return es >= 16 ? 2048 : 4096; }

static bool fused_ok(const void *src, size_t src_stride, const void *dst, size_t dst_stride,
                     size_t nchunks, size_t chunk_bytes, size_t es) {
  if (!(es == 2 || es == 4 || es == 8 || es == 16)) return false;
  if (chunk_bytes % es != 0) return false;
  const size_t count = chunk_bytes / es;
  if (count % fused_tile_elems(es) != 0) return false;
  if ((uintptr_t)src % 16 || (uintptr_t)dst % 16) return false;
  if (nchunks > 1 && (src_stride % 16 || dst_stride % 16)) return false;
  return true;
}

}  // namespace

// shared with mc_shuffle.hip
int mc_shuffle_impl(const void *src_, size_t src_stride, void *dst_, size_t dst_stride,
                    size_t nchunks, size_t chunk_bytes, size_t es, bool enc, int variant,
                    int max_blocks, const McBitRound *br, hipStream_t st);

extern "C" {

size_t mc_fletcher32_workspace(size_t nbytes) {
  return fused_partials_bytes(slices_for(nbytes, 1));  // >= partials_bytes(1, .)
}

int mc_fletcher32(const void *src, size_t nbytes, uint32_t *out_sum, void *workspace,
                  size_t workspace_bytes, mc_stream_t stream) {
  if (!out_sum || (!src && nbytes)) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (nbytes == 0) return mc_hip_status(hipMemsetAsync(out_sum, 0, sizeof(uint32_t), st));
  return f32_run(static_cast<const uint8_t *>(src), 0, nullptr, 0, 1, nbytes, F_SUM, out_sum,
                 workspace, workspace_bytes, st);
}

int mc_fletcher32_encode(const void *src, void *dst, size_t nbytes, void *workspace,
                         size_t workspace_bytes, mc_stream_t stream) {
  if (!src || !dst || nbytes == 0) return MC_EINVAL;
  return f32_run(static_cast<const uint8_t *>(src), 0, static_cast<uint8_t *>(dst), 0, 1, nbytes,
                 F_FOOTER, nullptr, workspace, workspace_bytes, (hipStream_t)stream);
}

int mc_fletcher32_encode_fused(const void *src, void *dst, size_t nbytes, void *workspace, size_t workspace_bytes,
                               uint32_t *ticket, mc_stream_t stream) {
  if (!ticket) return mc_fletcher32_encode(src, dst, nbytes, workspace, workspace_bytes, stream);
  if (!src || !dst || nbytes == 0 || (uintptr_t)ticket % 8) return MC_EINVAL;
  return f32_run(static_cast<const uint8_t *>(src), 0, static_cast<uint8_t *>(dst), 0, 1, nbytes, F_FOOTER, nullptr,
                 workspace, workspace_bytes, (hipStream_t)stream, ticket, 0);
}

int mc_fletcher32_verify(const void *src, size_t nbytes, uint32_t *out_pair, void *workspace,
                         size_t workspace_bytes, mc_stream_t stream) {
  if (!src || !out_pair || nbytes < 4) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const size_t payload = nbytes - 4;  // payload 0: checksum 0, footer still read
  return f32_run(static_cast<const uint8_t *>(src), 0, nullptr, 0, 1, payload, F_VERIFY, out_pair,
                 workspace, workspace_bytes, st);
}

int mc_fletcher32_verify_fused(const void *src, size_t nbytes, uint32_t *out_rec, uint32_t seq, void *workspace,
                               size_t workspace_bytes, uint32_t *ticket, mc_stream_t stream) {
  if (!ticket) {
    if (seq) return MC_EINVAL;  // the two-launch path publishes no sequence word
    return mc_fletcher32_verify(src, nbytes, out_rec, workspace, workspace_bytes, stream);
  }
  if ((uintptr_t)ticket % 8) return MC_EINVAL;
  if (!src || !out_rec || nbytes < 4) return MC_EINVAL;
  return f32_run(static_cast<const uint8_t *>(src), 0, nullptr, 0, 1, nbytes - 4, F_VERIFY, out_rec, workspace,
                 workspace_bytes, (hipStream_t)stream, ticket, seq);
}

int mc_fletcher32_batch(const void *src, size_t stride, size_t nchunks, size_t chunk_bytes,
                        uint32_t *out_sums, void *workspace, size_t workspace_bytes,
                        mc_stream_t stream) {
  if (nchunks == 0) return MC_OK;
  if (!src || !out_sums || (nchunks > 1 && stride < chunk_bytes)) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (chunk_bytes == 0) return mc_hip_status(hipMemsetAsync(out_sums, 0, nchunks * 4, st));
  return f32_run(static_cast<const uint8_t *>(src), stride, nullptr, 0, nchunks, chunk_bytes, F_SUM,
                 out_sums, workspace, workspace_bytes, st);
}

int mc_fletcher32_encode_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                               size_t nchunks, size_t chunk_bytes, void *workspace,
                               size_t workspace_bytes, mc_stream_t stream) {
  if (nchunks == 0) return MC_OK;
  if (!src || !dst || chunk_bytes == 0) return MC_EINVAL;
  if (nchunks > 1 && (src_stride < chunk_bytes || dst_stride < chunk_bytes + 4)) return MC_EINVAL;
  if (nchunks > 0x7fffffffu) return MC_EINVAL;
  return f32_run(static_cast<const uint8_t *>(src), src_stride, static_cast<uint8_t *>(dst), dst_stride,
                 nchunks, chunk_bytes, F_FOOTER, nullptr, workspace, workspace_bytes,
                 (hipStream_t)stream);
}

int mc_fletcher32_decode_batch(const void *src, size_t src_stride, void *dst, size_t dst_stride,
                               size_t nchunks, size_t encoded_bytes, uint32_t *out_pairs,
                               void *workspace, size_t workspace_bytes, mc_stream_t stream) {
  if (nchunks == 0) return MC_OK;
  if (!src || !out_pairs || encoded_bytes < 4) return MC_EINVAL;
  const size_t n = encoded_bytes - 4;
  if (nchunks > 1 && (src_stride < encoded_bytes || (dst && dst_stride < n))) return MC_EINVAL;
  if (nchunks > 0x7fffffffu) return MC_EINVAL;
  return f32_run(static_cast<const uint8_t *>(src), src_stride, n ? static_cast<uint8_t *>(dst) : nullptr,
                 dst_stride, nchunks, n, F_VERIFY, out_pairs, workspace, workspace_bytes,
                 (hipStream_t)stream);
}

size_t mc_fletcher32_batch_workspace(size_t nchunks, size_t chunk_bytes) {
  return partials_bytes(nchunks, slices_for(chunk_bytes, nchunks));
}

size_t mc_shuffle_fletcher32_workspace(size_t nchunks, size_t chunk_bytes, size_t elementsize) {
  // fused path: one partial per tile; fallback path: the standalone slices
  const size_t es = elementsize ? elementsize : 1;
  const size_t tiles = (es == 2 || es == 4 || es == 8 || es == 16) && chunk_bytes % es == 0
                           ? (chunk_bytes / es) / fused_tile_elems(es) + 1
                           : 1;
  const size_t a = nchunks * tiles * 3 * sizeof(uint32_t);
  const size_t b = partials_bytes(nchunks, slices_for(chunk_bytes, nchunks));
  return a > b ? a : b;
}

int mc_shuffle_fletcher32_encode_batch(const void *src, size_t src_stride, void *dst,
                                       size_t dst_stride, size_t nchunks, size_t chunk_bytes,
                                       size_t elementsize, void *workspace,
                                       size_t workspace_bytes, mc_stream_t stream) {
  if (nchunks == 0) return MC_OK;
  if (!src || !dst || chunk_bytes == 0) return MC_EINVAL;
  if (nchunks > 1 && (src_stride < chunk_bytes || dst_stride < chunk_bytes + 4)) return MC_EINVAL;
  if (workspace_bytes < mc_shuffle_fletcher32_workspace(nchunks, chunk_bytes, elementsize) || !workspace)
    return MC_ENOSPC;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  const size_t es = elementsize ? elementsize : 1;
  if (nchunks == 1) { src_stride = chunk_bytes; dst_stride = chunk_bytes + 4; }
  if (!fused_ok(src, src_stride, dst, dst_stride, nchunks, chunk_bytes, es)) {
    // two passes: shuffle into place, then checksum + footer over the result
    int rc = mc_shuffle_impl(src, src_stride, dst, dst_stride, nchunks, chunk_bytes, es, true, 0, 0,
                             nullptr, st);
    if (rc != MC_OK) return rc;
    const unsigned nsl = slices_for(chunk_bytes, nchunks);
    uint32_t *partials = static_cast<uint32_t *>(workspace);
    launch_partial(d, dst_stride, nullptr, 0, nchunks, chunk_bytes, nsl, partials, nullptr, F_SUM, nullptr, 0, st);
    rc = mc_last_launch();
    if (rc != MC_OK) return rc;
    k_f32_finalize<<<(unsigned)nchunks, MC_BLOCK, 0, st>>>(
        partials, nsl, nchunks, F_FOOTER, nullptr, 0, d, dst_stride, chunk_bytes, nullptr);
    return mc_last_launch();
  }
  ChunkMap m;
  m.count = chunk_bytes / es;
  m.tiles_per_chunk = m.count / fused_tile_elems(es);
  m.src_stride = src_stride;
  m.dst_stride = dst_stride;
  m.group = 1;
  const size_t ntiles = m.tiles_per_chunk * nchunks;
  uint32_t *partials = static_cast<uint32_t *>(workspace);
  switch (es) {
    case 2: k_shuffle_f32_enc<2, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
    case 4: k_shuffle_f32_enc<4, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
    case 8: k_shuffle_f32_enc<8, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
    default: k_shuffle_f32_enc<16, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
  }
  int rc = mc_last_launch();
  if (rc != MC_OK) return rc;
  k_f32_finalize<<<(unsigned)nchunks, MC_BLOCK, 0, st>>>(
      partials, (unsigned)m.tiles_per_chunk, nchunks, F_FOOTER, nullptr, 0, d, dst_stride,
      chunk_bytes, nullptr);
  return mc_last_launch();
}

int mc_fletcher32_unshuffle_batch(const void *src, size_t src_stride, void *dst,
                                  size_t dst_stride, size_t nchunks, size_t chunk_bytes,
                                  size_t elementsize, uint32_t *status, void *workspace,
                                  size_t workspace_bytes, mc_stream_t stream) {
  if (nchunks == 0) return MC_OK;
  if (!src || !dst || !status || chunk_bytes == 0) return MC_EINVAL;
  if (nchunks > 1 && (src_stride < chunk_bytes + 4 || dst_stride < chunk_bytes)) return MC_EINVAL;
  if (workspace_bytes < mc_shuffle_fletcher32_workspace(nchunks, chunk_bytes, elementsize) || !workspace)
    return MC_ENOSPC;
  hipStream_t st = (hipStream_t)stream;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  const size_t es = elementsize ? elementsize : 1;
  if (nchunks == 1) { src_stride = chunk_bytes + 4; dst_stride = chunk_bytes; }
  if (!fused_ok(src, src_stride, dst, dst_stride, nchunks, chunk_bytes, es)) {
    // two passes: verify over the payloads, then unshuffle
    int rc = f32_run(s, src_stride, nullptr, 0, nchunks, chunk_bytes, F_VERIFY, status, workspace,
                     workspace_bytes, st);
    if (rc != MC_OK) return rc;
    return mc_shuffle_impl(src, src_stride, dst, dst_stride, nchunks, chunk_bytes, es, false, 0, 0,
                           nullptr, st);
  }
  ChunkMap m;
  m.count = chunk_bytes / es;
  m.tiles_per_chunk = m.count / fused_tile_elems(es);
  m.src_stride = src_stride;
  m.dst_stride = dst_stride;
  m.group = 1;
  const size_t ntiles = m.tiles_per_chunk * nchunks;
  uint32_t *partials = static_cast<uint32_t *>(workspace);
  switch (es) {
    case 2: k_f32_unshuffle<2, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
    case 4: k_f32_unshuffle<4, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
    case 8: k_f32_unshuffle<8, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
    default: k_f32_unshuffle<16, true><<<(unsigned)ntiles, MC_BLOCK, 0, st>>>(s, d, m, partials); break;
  }
  int rc = mc_last_launch();
  if (rc != MC_OK) return rc;
  k_f32_finalize<<<(unsigned)nchunks, MC_BLOCK, 0, st>>>(
      partials, (unsigned)m.tiles_per_chunk, nchunks, F_VERIFY, s, src_stride, nullptr, 0,
      chunk_bytes, status);
  return mc_last_launch();
}

}  // extern "C"
