// lab_scan1p.hip -- LAB ONLY (libmcodec_lab.so): single-pass, one-read
// decodes of the integer scans, measured against the product's three-pass
// scans and rejected this round ("Single-pass scans"):
//   * same-width integer Delta decode, np.cumsum(enc, out=dec) with
//     astype == dtype of 1, 2 or 4 bytes (delta.py:69-83);
//   * the fused FixedScaleOffset <- Delta <- Shuffle decode of a Zarr filter
//     chain [FixedScaleOffset(f4|f8 -> i2|u2|i4|u4), Delta] + Shuffle
//     (fixedscaleoffset.py:99-113, delta.py:69-83, _shuffle.pyx:23-30).
//
// The three-pass scan (tile totals, scan of the totals, rescan + store) reads
// the encoded bytes twice: 3N of HBM traffic for the 2N a decode needs.  Here
// a persistent grid takes PARTITIONS of 32-64 KiB of encoded bytes by atomic
// ticket (mc_lookback.h) and keeps each one on chip from its read to its
// write, software-pipelined one partition deep:
//   stage(p)   the partition's bytes (already in registers) are scanned unit
//              by unit (a unit = one 16-B vector per byte plane); the units'
//              local inclusive scans go to LDS, one multi-value block scan
//              of the unit totals gives every unit its offset in the
//              partition and the partition's aggregate, which is published;
//   then, per iteration:
//     poll     the first look-back round for p (1024 status words, one
//              block-wide read) is issued BEFORE ...
//     load(q)  ... the next partition's loads (lane-contiguous 16-B
//              nontemporal loads, every one of a thread's loads in flight),
//              so the look-back's latency hides under them;
//     resolve  the exclusive prefix of p (decoupled look-back: predecessors
//              hold earlier tickets, so they are running or done);
//     emit(p)  every output vector = prefix + unit offset + local scan, read
//              back from LDS in the store-friendly order (lane-contiguous
//              16-B nontemporal stores) -- while q's loads land;
//     stage(q).
// HBM traffic is the algorithmic N_in + N_out; the encoded bytes are read
// once.  Arithmetic is modular (mod 2^(8*itemsize)), exactly numpy's wrapping
// integer add, so the result is bit-exact whatever the partitioning.
#include <type_traits>

#include "mc_c4.h"
#include "lab_lookback.h"

namespace {

// ---------------------------------------------------------------------------
// shared pieces
// ---------------------------------------------------------------------------
template <int ES>
using lt_t = typename std::conditional<ES == 1, uint8_t, typename std::conditional<ES == 2, uint16_t, uint32_t>::type>::type;

// c + x for every ES-byte lane of the dword x, mod 2^(8*ES) per lane
template <int ES>
MC_DEV uint32_t swar_add(uint32_t x, uint32_t c) {
  if constexpr (ES == 4) {
    return x + c;
  } else if constexpr (ES == 2) {
    return ((x + c) & 0xffffu) | ((x & 0xffff0000u) + (c << 16));
  } else {
    const uint32_t c4 = (c & 0xffu) * 0x01010101u;
    return ((x & 0x7f7f7f7fu) + (c4 & 0x7f7f7f7fu)) ^ ((x ^ c4) & 0x80808080u);
  }
}

// Prefix of a partition when its look-back times out (guard only: with
// ticket order a predecessor is always running): the sum of every delta
// before it, read from the data itself; counted in workspace word [2].
// `sum_unit(j)` is the delta sum of unit j.
template <class F>
MC_DEV uint32_t lb_prefix_from_data(size_t nunits, F sum_unit, uint32_t *red) {
  uint32_t acc = 0;
  for (size_t j = threadIdx.x; j < nunits; j += MC_BLOCK) acc += sum_unit(j);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < MC_BLOCK / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

// Unit offsets of a staged partition into seg[] (unit j = k*MC_BLOCK + tid)
// from the per-thread unit totals; returns the partition aggregate.
template <int UPT, typename T>
MC_DEV uint32_t stage_offsets(const uint32_t (&tot)[UPT], T *seg, uint32_t (*red)[MC_BLOCK / 64]) {
  uint32_t ex[UPT], tk[UPT];
  mc_block_excl_scan_multi<UPT>(tot, ex, tk, red);
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    seg[k * MC_BLOCK + threadIdx.x] = (T)(run + ex[k]);
    run += tk[k];
  }
  return run;
}

// The partition loop shared by both decodes.  Two LDS partition buffers;
// per iteration, with p staged in buffer b (aggregate published) and the
// ticket q already taken:
//   poll(p)        first look-back round for p (1024 status words), issued
//                  BEFORE q's loads so that waiting for it never waits for them
//   load(q)        every load of q in flight
//   stage(q, b^1)  unit scans to LDS, offsets, aggregate -> published: a
//                  partition's aggregate appears one load + stage after its
//                  ticket, whatever else its workgroup is doing, so look-backs
//                  never queue behind another workgroup's emit (a convoy)
//   resolve(p)     the rest of p's look-back; its inclusive prefix published
//   emit(p, b)     the output of p
//   ticket         the next partition, and the buffers swap.
// Pol provides:
//   Raw                               registers holding one partition's bytes
//   load(raw, part)                   issue the partition's loads
//   stage(raw, part, sm, buf) -> agg  unit scans + offsets into buffer buf
//   emit(part, prefix, sm, buf)       the partition's output from buffer buf
//   sum_unit(j), units_before(part)   the guard path's data-derived prefix
// `trace` (lab measurement only, NULL in the product): per partition, thread
// 0 records wall_clock64() at ticket, staged (aggregate published), look-back
// resolved, emitted, and the workgroup id.
template <class Pol>
MC_DEV void scan1p_loop(const Pol &pol, typename Pol::Smem &sm, uint32_t *ws, size_t npart, unsigned spins,
                        uint64_t *trace) {
  uint64_t *status = reinterpret_cast<uint64_t *>(ws + 4);
  auto mark = [&](size_t part, int what) {
    if (trace && threadIdx.x == 0) trace[8 * part + what] = wall_clock64();
  };
  if (threadIdx.x == 0) sm.slot = atomicAdd(ws, 1u);
  __syncthreads();
  size_t p = sm.slot;
  __syncthreads();
  if (p < npart) {
    typename Pol::Raw raw;
    int b = 0;
    mark(p, 0);
    if (trace && threadIdx.x == 0) trace[8 * p + 5] = blockIdx.x;
    pol.load(raw, p);
    uint32_t agg = pol.stage(raw, p, sm, b);
    if (threadIdx.x == 0) {
      if (p == 0) mc_lb_publish_inclusive(status, 0, agg);
      else mc_lb_publish_aggregate(status, p, agg);
      mark(p, 1);
      sm.slot = atomicAdd(ws, 1u);
    }
    __syncthreads();
    size_t q = sm.slot;
    for (;;) {
      uint64_t sw[4];
      mc_lb_block_poll(status, (long long)p - 1, sw);
      __builtin_amdgcn_sched_barrier(0);  // the polls stay ahead of q's loads
      uint32_t agg_q = 0;
      if (q < npart) {
        mark(q, 0);
        if (trace && threadIdx.x == 0) trace[8 * q + 5] = blockIdx.x;
        pol.load(raw, q);
        agg_q = pol.stage(raw, q, sm, b ^ 1);
        if (threadIdx.x == 0) mc_lb_publish_aggregate(status, q, agg_q);
        mark(q, 1);
      }
      mark(p, 2);
      bool ok;
      uint32_t pre = mc_lb_block_lookback(status, p, agg, sw, spins, ok, sm.lb);
      if (!ok) {
        pre = lb_prefix_from_data(pol.units_before(p), [&](size_t j) { return pol.sum_unit(j); }, sm.red[0]);
        if (threadIdx.x == 0) {
          mc_lb_publish_inclusive(status, p, pre + agg);
          atomicAdd(&ws[2], 1u);
        }
      }
      mark(p, 3);
      pol.emit(p, pre, sm, b);
      mark(p, 4);
      if (q >= npart) break;
      if (threadIdx.x == 0) sm.slot = atomicAdd(ws, 1u);
      __syncthreads();  // emit's LDS reads of buffer b are done before the next stage reuses it
      p = q;
      agg = agg_q;
      b ^= 1;
      q = sm.slot;
      __syncthreads();  // everyone has read the ticket before thread 0 overwrites the slot
    }
  }
  mc_lb_retire(ws, npart, &sm.slot);
}

// ---------------------------------------------------------------------------
// same-width integer Delta decode: a unit is one 16-B vector (16/ES elements)
// ---------------------------------------------------------------------------
template <int ES>
constexpr int d1p_units() { return ES == 4 ? 1024 : 2048; }  // 16 / 32 KiB partitions, two in LDS

template <int ES>
MC_DEV uint32_t unit_total(mc_u32x4 w) {
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (ES == 1) a = __builtin_amdgcn_udot4(w[i], 0x01010101u, a, false);
    else if constexpr (ES == 2) a += (w[i] & 0xffffu) + (w[i] >> 16);
    else a += w[i];
  }
  return a;
}

// inclusive scan of the ES-byte lanes of one 16-B unit, mod 2^(8*ES) per lane
template <int ES>
MC_DEV mc_u32x4 unit_scan(mc_u32x4 w, uint32_t &total) {
  uint32_t d[4] = {w.x, w.y, w.z, w.w};
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t x = d[i];
    if constexpr (ES == 1) {  // bytes: two SWAR doubling steps inside the dword
      x = ((x & 0x7f7f7f7fu) + ((x << 8) & 0x7f7f7f7fu)) ^ ((x ^ (x << 8)) & 0x80808080u);
      x = ((x & 0x7f7f7f7fu) + ((x << 16) & 0x7f7f7f7fu)) ^ ((x ^ (x << 16)) & 0x80808080u);
    } else if constexpr (ES == 2) {
      x = x + (x << 16);  // high half += low half (mod 2^16 by the shift)
    }
    x = swar_add<ES>(x, carry);
    carry = ES == 4 ? x : (x >> (32 - 8 * ES));
    d[i] = x;
  }
  total = carry;
  return mc_u32x4{d[0], d[1], d[2], d[3]};
}

template <int ES>
struct DeltaPol {
  static constexpr int P = d1p_units<ES>();
  static constexpr int UPT = P / MC_BLOCK;
  using T = lt_t<ES>;
  struct Raw {
    mc_u32x4 w[UPT];
  };
  struct Smem {
    mc_u32x4 loc[2][P];  // local inclusive scans, unit by unit
    T seg[2][P];         // unit offsets within the partition
    uint32_t red[UPT][MC_BLOCK / 64];
    McLbBlock lb;
    uint32_t slot;
  };
  const mc_u32x4 *s16;
  mc_u32x4 *d16;
  size_t nunits;

  MC_DEV void load(Raw &r, size_t part) const {
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const size_t u = part * P + (size_t)k * MC_BLOCK + threadIdx.x;
      r.w[k] = u < nunits ? __builtin_nontemporal_load(s16 + u) : mc_u32x4{0, 0, 0, 0};
    }
  }
  MC_DEV uint32_t stage(const Raw &r, size_t, Smem &sm, int b) const {
    uint32_t tot[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) sm.loc[b][k * MC_BLOCK + threadIdx.x] = unit_scan<ES>(r.w[k], tot[k]);
    return stage_offsets<UPT, T>(tot, sm.seg[b], sm.red);
  }
  MC_DEV void emit(size_t part, uint32_t pre, Smem &sm, int b) const {
#pragma unroll 4
    for (int k = 0; k < UPT; ++k) {
      const int j = k * MC_BLOCK + threadIdx.x;
      const size_t u = part * P + j;
      if (u >= nunits) break;
      const uint32_t c = pre + (uint32_t)sm.seg[b][j];
      const mc_u32x4 l = sm.loc[b][j];
      __builtin_nontemporal_store(mc_u32x4{swar_add<ES>(l.x, c), swar_add<ES>(l.y, c), swar_add<ES>(l.z, c),
                                           swar_add<ES>(l.w, c)},
                                  d16 + u);
    }
  }
  MC_DEV uint32_t sum_unit(size_t j) const { return unit_total<ES>(__builtin_nontemporal_load(s16 + j)); }
  MC_DEV size_t units_before(size_t part) const { return part * P; }
};

template <int ES>
__global__ __launch_bounds__(MC_BLOCK) void k_delta_dec1p(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t nunits_total,
                                                         uint32_t *ws, size_t npart, unsigned spins,
                                                         uint64_t *trace) {
  __shared__ __attribute__((aligned(16))) typename DeltaPol<ES>::Smem sm;
  DeltaPol<ES> pol;
  pol.s16 = reinterpret_cast<const mc_u32x4 *>(src);
  pol.d16 = reinterpret_cast<mc_u32x4 *>(dst);
  pol.nunits = nunits_total;
  scan1p_loop(pol, sm, ws, npart, spins, trace);
}

// VE consecutive T values from LDS as ONE vector read (16, 8 or 4 B)
template <typename T, int VE>
MC_DEV void lds_read_run(const T *p, uint32_t (&l)[VE]) {
  constexpr int B = VE * (int)sizeof(T);
  if constexpr (B == 16) {
    const mc_u32x4 v = *reinterpret_cast<const mc_u32x4 *>(p);
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < VE; ++i) l[i] = d[i];
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) l[i] = (d[i / 2] >> (16 * (i & 1))) & 0xffffu;
    }
  } else if constexpr (B == 8) {
    const mc_u32x2 v = *reinterpret_cast<const mc_u32x2 *>(p);
    const uint32_t d[2] = {v.x, v.y};
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < VE; ++i) l[i] = d[i];
    } else {
#pragma unroll
      for (int i = 0; i < VE; ++i) l[i] = (d[i / 2] >> (16 * (i & 1))) & 0xffffu;
    }
  } else {
    static_assert(B == 4 && sizeof(T) == 2, "unsupported run");
    const uint32_t d = *reinterpret_cast<const uint32_t *>(p);
    l[0] = d & 0xffffu;
    l[1] = d >> 16;
  }
}

// ---------------------------------------------------------------------------
// FSO <- Delta <- Shuffle(ES): a unit is 16 elements (one 16-B vector per
// byte plane); the local scans are kept at the astype width, element by
// element, so the store side can read any run of consecutive elements.
// ---------------------------------------------------------------------------
template <int A>
constexpr int c41p_elems() { return c4_es<A>() == 2 ? 16384 : 8192; }  // 32 KiB of local scans, two in LDS

template <int D, int A>
struct C4Pol {
  static constexpr int ES = c4_es<A>();
  static constexpr int E = c41p_elems<A>();
  static constexpr int UNITS = E / 16;
  static constexpr int UPT = UNITS / MC_BLOCK;
  static constexpr int DS = D == MC_F4 ? 4 : 8;
  static constexpr int VE = 16 / DS;  // output elements per 16-B store
  using T = lt_t<ES>;
  struct Raw {
    mc_u32x4 pl[UPT][ES];
  };
  struct Smem {
    T loc[2][E];
    T seg[2][UNITS];
    uint32_t red[UPT][MC_BLOCK / 64];
    McLbBlock lb;
    uint32_t slot;
  };
  const uint8_t *src;
  uint8_t *dst;
  C4Params p;

  MC_DEV void load(Raw &r, size_t part) const {
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const size_t e0 = part * E + 16 * ((size_t)k * MC_BLOCK + threadIdx.x);
#pragma unroll
      for (int b = 0; b < ES; ++b)
        r.pl[k][b] = e0 < p.n ? mc_ld16<true>(src + (size_t)b * p.n + e0) : mc_u32x4{0, 0, 0, 0};
    }
  }
  MC_DEV uint32_t stage(const Raw &r, size_t, Smem &sm, int b) const {
    uint32_t tot[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      uint32_t v[C4_PER];
      c4_planes_to_deltas<A, ES>(r.pl[k], v);
      uint32_t run = 0;
#pragma unroll
      for (int i = 0; i < C4_PER; ++i) {
        run += v[i];
        v[i] = run;
      }
      tot[k] = run;
      mc_u32x4 *d4 = reinterpret_cast<mc_u32x4 *>(sm.loc[b] + 16 * (k * MC_BLOCK + threadIdx.x));
      if constexpr (ES == 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
          d4[h] = mc_u32x4{(v[8 * h] & 0xffffu) | (v[8 * h + 1] << 16), (v[8 * h + 2] & 0xffffu) | (v[8 * h + 3] << 16),
                           (v[8 * h + 4] & 0xffffu) | (v[8 * h + 5] << 16), (v[8 * h + 6] & 0xffffu) | (v[8 * h + 7] << 16)};
      } else {
#pragma unroll
        for (int h = 0; h < 4; ++h) d4[h] = mc_u32x4{v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
      }
    }
    return stage_offsets<UPT, T>(tot, sm.seg[b], sm.red);
  }
  MC_DEV void emit(size_t part, uint32_t pre, Smem &sm, int b) const {
    const size_t e_base = part * E;
#pragma unroll 4
    for (int r = 0; r < E / VE / MC_BLOCK; ++r) {
      const int e = VE * (r * MC_BLOCK + (int)threadIdx.x);
      if (e_base + e >= p.n) break;
      const uint32_t c = pre + (uint32_t)sm.seg[b][e / 16];
      uint32_t l[VE];
      lds_read_run<T, VE>(sm.loc[b] + e, l);
      uint32_t o[4];
#pragma unroll
      for (int i = 0; i < VE; ++i) {
        const uint64_t x = fso_dec<D, A>(mc_wrap((int64_t)(uint32_t)(c + l[i]), A), p);
        if constexpr (DS == 4) {
          o[i] = (uint32_t)x;
        } else {
          o[2 * i] = (uint32_t)x;
          o[2 * i + 1] = (uint32_t)(x >> 32);
        }
      }
      mc_st16<true>(dst + (e_base + e) * DS, mc_u32x4{o[0], o[1], o[2], o[3]});
    }
  }
  MC_DEV uint32_t sum_unit(size_t j) const {
    uint32_t v[C4_PER];
    load16_deltas<A, ES>(src, p.n, 16 * j, v);
    uint32_t a = 0;
#pragma unroll
    for (int i = 0; i < C4_PER; ++i) a += v[i];
    return a;
  }
  MC_DEV size_t units_before(size_t part) const { return part * (E / 16); }
};

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_dec1p(const uint8_t *__restrict__ src,
                                                      uint8_t *__restrict__ dst, uint32_t *ws, size_t npart,
                                                      C4Params p, unsigned spins, uint64_t *trace) {
  __shared__ __attribute__((aligned(16))) typename C4Pol<D, A>::Smem sm;
  C4Pol<D, A> pol;
  pol.src = src;
  pol.dst = dst;
  pol.p = p;
  scan1p_loop(pol, sm, ws, npart, spins, trace);
}

// persistent grid: enough workgroups to fill every CU at the occupancy the
// kernel's LDS and registers allow (tickets make correctness independent of it)
template <typename K>
static unsigned resident_grid(K kernel, size_t npart) {
  int dev = 0, cus = 256, per_cu = 1;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, MC_BLOCK, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const size_t g = (size_t)cus * (size_t)per_cu;
  return (unsigned)(npart < g ? npart : g);
}

template <int D, int A>
static void launch_c4_dec1p(const uint8_t *s, uint8_t *d, uint32_t *ws, const C4Params &p, unsigned spins,
                            uint64_t *trace, hipStream_t st) {
  const size_t npart = (p.n + c41p_elems<A>() - 1) / c41p_elems<A>();
  static const unsigned cap = resident_grid(k_c4_dec1p<D, A>, ~(size_t)0 >> 1);
  const unsigned grid = (unsigned)(npart < cap ? npart : cap);
  k_c4_dec1p<D, A><<<grid, MC_BLOCK, 0, st>>>(s, d, ws, npart, p, spins, trace);
}

}  // namespace

// ---------------------------------------------------------------------------
// host entry points (C++ linkage; the C ABI wrappers live in mc_scan.hip and
// mc_c4.hip)
// ---------------------------------------------------------------------------
size_t mc_delta_dec1p_state_bytes(size_t n, int es) {
  if (!(es == 1 || es == 2 || es == 4)) return 0;
  const size_t units = n * (size_t)es / 16;
  const size_t P = es == 4 ? (size_t)d1p_units<4>() : (size_t)d1p_units<1>();  // units per partition
  return mc_lb_ws_bytes((units + P - 1) / P);
}

// dst = cumsum(src) in the same width es (1, 2, 4); n * es % 16 == 0, 16-B
// aligned buffers, `state` = mc_delta_dec1p_state_bytes(n, es) zeroed bytes
// (left zeroed by the call).  Returns MC_EINVAL when the shape does not fit.
// `spins` bounds each look-back wait (MC_LB_WAVE_SPINS; the lab passes 0 to
// force the data-derived prefix wherever a predecessor is not yet published).
int mc_delta_dec1p(const void *src, void *dst, size_t n, int es, void *state, hipStream_t st,
                   unsigned spins, uint64_t *trace) {
  if (!(es == 1 || es == 2 || es == 4) || (n * (size_t)es) % 16 != 0) return MC_EINVAL;
  if ((uintptr_t)src % 16 || (uintptr_t)dst % 16 || (uintptr_t)state % 16) return MC_EINVAL;
  const size_t units = n * (size_t)es / 16;
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint32_t *ws = static_cast<uint32_t *>(state);
  switch (es) {
    case 1: {
      const size_t npart = (units + d1p_units<1>() - 1) / d1p_units<1>();
      static const unsigned cap = resident_grid(k_delta_dec1p<1>, ~(size_t)0 >> 1);
      k_delta_dec1p<1><<<(unsigned)(npart < cap ? npart : cap), MC_BLOCK, 0, st>>>(s, d, units, ws, npart,
                                                                                  spins, trace);
      break;
    }
    case 2: {
      const size_t npart = (units + d1p_units<2>() - 1) / d1p_units<2>();
      static const unsigned cap = resident_grid(k_delta_dec1p<2>, ~(size_t)0 >> 1);
      k_delta_dec1p<2><<<(unsigned)(npart < cap ? npart : cap), MC_BLOCK, 0, st>>>(s, d, units, ws, npart,
                                                                                  spins, trace);
      break;
    }
    default: {
      const size_t npart = (units + d1p_units<4>() - 1) / d1p_units<4>();
      static const unsigned cap = resident_grid(k_delta_dec1p<4>, ~(size_t)0 >> 1);
      k_delta_dec1p<4><<<(unsigned)(npart < cap ? npart : cap), MC_BLOCK, 0, st>>>(s, d, units, ws, npart,
                                                                                  spins, trace);
      break;
    }
  }
  return mc_last_launch();
}

size_t mc_c4_dec1p_state_bytes(size_t n, int astype) {
  const size_t E = (astype == MC_I2 || astype == MC_U2) ? (size_t)c41p_elems<MC_I2>() : (size_t)c41p_elems<MC_I4>();
  return mc_lb_ws_bytes((n + E - 1) / E);
}

// the fused FSO <- Delta <- Shuffle decode (c4_ok shapes), single pass;
// `state` = mc_c4_dec1p_state_bytes(n, astype) zeroed bytes
int mc_c4_dec1p(const void *src, void *dst, size_t n, int astype, int dtype, double scale, double offset,
                void *state, hipStream_t st, unsigned spins, uint64_t *trace) {
  if (!c4_ok(src, dst, n, dtype, astype) || (uintptr_t)state % 16) return MC_EINVAL;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint32_t *ws = static_cast<uint32_t *>(state);
  MC_C4_DISPATCH(launch_c4_dec1p, s, d, ws, p, spins, trace, st);
  return mc_last_launch();
}
