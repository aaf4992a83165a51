// mc_scan1p.hip -- one-launch, one-read decodes of the integer scans:
//   * same-width integer Delta decode, np.cumsum(enc, out=dec) with
//     astype == dtype of 1, 2 or 4 bytes (delta.py:69-83);
//   * the fused FixedScaleOffset <- Delta <- Shuffle decode of a Zarr filter
//     chain [FixedScaleOffset(f4|f8 -> i2|u2|i4|u4), Delta] + Shuffle
//     (fixedscaleoffset.py:99-113, delta.py:69-83, _shuffle.pyx:23-30).
//
// The three-pass scan (tile totals, scan of the totals, rescan + store) reads
// the encoded bytes twice: 3N of HBM traffic for the 2N a decode needs.  Here
// a persistent grid takes PARTITIONS of 64 KiB of encoded bytes by atomic
// ticket (mc_lookback.h) and keeps each one in LDS from its read to its
// write:
//   1. stream the partition in (lane-contiguous 16-B nontemporal loads, all
//      of a thread's loads in flight at once), scan every 16-B unit in
//      registers and park the unit's local inclusive scans in LDS;
//   2. one multi-value block scan of the unit totals gives every unit its
//      offset inside the partition and the partition's aggregate;
//   3. one wave publishes the aggregate and looks back over its predecessors'
//      status words (decoupled look-back; predecessors hold earlier tickets,
//      so they are running or done) for the exclusive prefix;
//   4. every output vector = prefix + unit offset + local scan, read back from
//      LDS in the store-friendly order (lane-contiguous 16-B stores).
// HBM traffic is the algorithmic N_in + N_out; the encoded bytes are read
// once.  Arithmetic is modular (mod 2^(8*itemsize)), exactly numpy's wrapping
// integer add, so the result is bit-exact whatever the partitioning.
#include <type_traits>

#include "mc_c4.h"
#include "mc_lookback.h"

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

// Partition prefix when a look-back round times out: the sum of every delta
// before `e_base`, read from the data itself (correct under any schedule;
// counted in workspace word [2]).  `sum_units` adds the deltas of the 16-B
// units [0, nunits) in the block's threads.
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

// Steps 2-3 for one partition: unit offsets into seg[], the exclusive prefix
// of the partition into *pre_slot.  Every thread calls it.
template <int UPT, typename T, class F>
MC_DEV void partition_prefix(const uint32_t (&tot)[UPT], T *seg, uint64_t *status, uint32_t *ws, size_t part,
                             size_t units_before, F sum_unit, uint32_t (*red)[MC_BLOCK / 64], uint32_t *pre_slot,
                             uint32_t *ok_slot, unsigned spins) {
  uint32_t ex[UPT], tk[UPT];
  mc_block_excl_scan_multi<UPT>(tot, ex, tk, red);
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    seg[k * MC_BLOCK + threadIdx.x] = (T)(run + ex[k]);
    run += tk[k];
  }
  const uint32_t agg = run;
  if (threadIdx.x < 64) {
    bool ok;
    const uint32_t pre = mc_lb_lookback_wave4<false>(status, part, agg, ok, spins);
    if (threadIdx.x == 0) {
      *pre_slot = pre;
      *ok_slot = ok;
    }
  }
  __syncthreads();
  if (!*ok_slot) {  // guard only: a predecessor did not publish within the spin bound
    const uint32_t pre = lb_prefix_from_data(units_before, sum_unit, red[0]);
    if (threadIdx.x == 0) {
      *pre_slot = pre;
      mc_lb_publish_inclusive(status, part, pre + agg);
      atomicAdd(&ws[2], 1u);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// same-width integer Delta decode: a unit is one 16-B vector (16/ES elements)
// ---------------------------------------------------------------------------
template <int ES>
constexpr int d1p_units() { return ES == 4 ? 2048 : 4096; }  // 32 / 64 KiB partitions

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
__global__ __launch_bounds__(MC_BLOCK) void k_delta_dec1p(const uint8_t *__restrict__ src,
                                                         uint8_t *__restrict__ dst, size_t nunits_total,
                                                         uint32_t *ws, size_t npart, unsigned spins) {
  constexpr int P = d1p_units<ES>();
  constexpr int UPT = P / MC_BLOCK;
  using T = lt_t<ES>;
  __shared__ __attribute__((aligned(16))) mc_u32x4 loc[P];  // local inclusive scans, unit by unit
  __shared__ __attribute__((aligned(16))) T seg[P];         // unit offsets within the partition
  __shared__ uint32_t red[UPT][MC_BLOCK / 64];
  __shared__ uint32_t slot, pre_slot, ok_slot;
  uint64_t *status = reinterpret_cast<uint64_t *>(ws + 4);
  const mc_u32x4 *s16 = reinterpret_cast<const mc_u32x4 *>(src);
  mc_u32x4 *d16 = reinterpret_cast<mc_u32x4 *>(dst);
  for (;;) {
    const size_t part = mc_lb_ticket(ws, &slot);
    if (part >= npart) break;
    const size_t u_base = part * P;
    // 1. all of this thread's loads in flight, then the per-unit scans
    mc_u32x4 w[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const size_t u = u_base + (size_t)k * MC_BLOCK + threadIdx.x;
      w[k] = u < nunits_total ? __builtin_nontemporal_load(s16 + u) : mc_u32x4{0, 0, 0, 0};
    }
    uint32_t tot[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) loc[k * MC_BLOCK + threadIdx.x] = unit_scan<ES>(w[k], tot[k]);
    // 2-3. unit offsets, aggregate, look-back
    auto sum_unit = [&](size_t j) { return unit_total<ES>(__builtin_nontemporal_load(s16 + j)); };
    partition_prefix<UPT, T>(tot, seg, status, ws, part, u_base, sum_unit, red, &pre_slot, &ok_slot, spins);
    const uint32_t pre = pre_slot;
    // 4. output: unit j = prefix + seg[j] + its local scans
#pragma unroll 4
    for (int k = 0; k < UPT; ++k) {
      const int j = k * MC_BLOCK + threadIdx.x;
      const size_t u = u_base + j;
      if (u >= nunits_total) break;
      const uint32_t c = pre + (uint32_t)seg[j];
      const mc_u32x4 l = loc[j];
      __builtin_nontemporal_store(mc_u32x4{swar_add<ES>(l.x, c), swar_add<ES>(l.y, c), swar_add<ES>(l.z, c),
                                           swar_add<ES>(l.w, c)},
                                  d16 + u);
    }
    __syncthreads();  // loc / seg are refilled by the next partition
  }
  mc_lb_retire(ws, npart, &slot);
}

// VE consecutive T values from LDS as ONE vector read (8 or 16 B, or 4 B)
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
constexpr int c41p_elems() { return c4_es<A>() == 2 ? 32768 : 16384; }  // 64 KiB of local scans

template <int D, int A>
__global__ __launch_bounds__(MC_BLOCK) void k_c4_dec1p(const uint8_t *__restrict__ src,
                                                      uint8_t *__restrict__ dst, uint32_t *ws, size_t npart,
                                                      C4Params p, unsigned spins) {
  constexpr int ES = c4_es<A>();
  constexpr int E = c41p_elems<A>();
  constexpr int UNITS = E / 16;
  constexpr int UPT = UNITS / MC_BLOCK;
  constexpr int DS = D == MC_F4 ? 4 : 8;
  constexpr int VE = 16 / DS;  // output elements per 16-B store
  using T = lt_t<ES>;
  __shared__ __attribute__((aligned(16))) T loc[E];
  __shared__ __attribute__((aligned(16))) T seg[UNITS];
  __shared__ uint32_t red[UPT][MC_BLOCK / 64];
  __shared__ uint32_t slot, pre_slot, ok_slot;
  uint64_t *status = reinterpret_cast<uint64_t *>(ws + 4);
  for (;;) {
    const size_t part = mc_lb_ticket(ws, &slot);
    if (part >= npart) break;
    const size_t e_base = part * E;
    // 1. every plane vector of this thread's units in flight at once
    mc_u32x4 pl[UPT][ES];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const size_t e0 = e_base + 16 * ((size_t)k * MC_BLOCK + threadIdx.x);
#pragma unroll
      for (int b = 0; b < ES; ++b)
        pl[k][b] = e0 < p.n ? mc_ld16<true>(src + (size_t)b * p.n + e0) : mc_u32x4{0, 0, 0, 0};
    }
    uint32_t tot[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      uint32_t v[C4_PER];
      c4_planes_to_deltas<A, ES>(pl[k], v);
      uint32_t run = 0;
#pragma unroll
      for (int i = 0; i < C4_PER; ++i) {
        run += v[i];
        v[i] = run;
      }
      tot[k] = run;
      mc_u32x4 *dst4 = reinterpret_cast<mc_u32x4 *>(loc + 16 * (k * MC_BLOCK + threadIdx.x));
      if constexpr (ES == 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
          dst4[h] = mc_u32x4{(v[8 * h] & 0xffffu) | (v[8 * h + 1] << 16), (v[8 * h + 2] & 0xffffu) | (v[8 * h + 3] << 16),
                             (v[8 * h + 4] & 0xffffu) | (v[8 * h + 5] << 16), (v[8 * h + 6] & 0xffffu) | (v[8 * h + 7] << 16)};
      } else {
#pragma unroll
        for (int h = 0; h < 4; ++h) dst4[h] = mc_u32x4{v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]};
      }
    }
    // 2-3. unit offsets, aggregate, look-back
    auto sum_unit = [&](size_t j) {
      uint32_t v[C4_PER];
      load16_deltas<A, ES>(src, p.n, 16 * j, v);
      uint32_t a = 0;
#pragma unroll
      for (int i = 0; i < C4_PER; ++i) a += v[i];
      return a;
    };
    partition_prefix<UPT, T>(tot, seg, status, ws, part, e_base / 16, sum_unit, red, &pre_slot, &ok_slot, spins);
    const uint32_t pre = pre_slot;
    // 4. output vectors: VE consecutive elements per lane, lane-contiguous
#pragma unroll 4
    for (int r = 0; r < E / VE / MC_BLOCK; ++r) {
      const int e = VE * (r * MC_BLOCK + (int)threadIdx.x);
      if (e_base + e >= p.n) break;
      const uint32_t c = pre + (uint32_t)seg[e / 16];
      uint32_t l[VE];
      lds_read_run<T, VE>(loc + e, l);
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
    __syncthreads();  // loc / seg are refilled by the next partition
  }
  mc_lb_retire(ws, npart, &slot);
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
                            hipStream_t st) {
  const size_t npart = (p.n + c41p_elems<A>() - 1) / c41p_elems<A>();
  static const unsigned cap = resident_grid(k_c4_dec1p<D, A>, ~(size_t)0 >> 1);
  const unsigned grid = (unsigned)(npart < cap ? npart : cap);
  k_c4_dec1p<D, A><<<grid, MC_BLOCK, 0, st>>>(s, d, ws, npart, p, spins);
}

}  // namespace

// ---------------------------------------------------------------------------
// host entry points (C++ linkage; the C ABI wrappers live in mc_scan.hip and
// mc_c4.hip)
// ---------------------------------------------------------------------------
size_t mc_delta_dec1p_state_bytes(size_t n, int es) {
  if (!(es == 1 || es == 2 || es == 4)) return 0;
  const size_t units = n * (size_t)es / 16;
  const size_t P = es == 4 ? (size_t)d1p_units<4>() : (size_t)d1p_units<1>();
  return mc_lb_ws_bytes((units + P - 1) / P);
}

// dst = cumsum(src) in the same width es (1, 2, 4); n * es % 16 == 0, 16-B
// aligned buffers, `state` = mc_delta_dec1p_state_bytes(n, es) zeroed bytes
// (left zeroed by the call).  Returns MC_EINVAL when the shape does not fit.
// `spins` bounds each look-back wait (MC_LB_WAVE_SPINS; the lab passes 0 to
// force the data-derived prefix wherever a predecessor is not yet published).
int mc_delta_dec1p(const void *src, void *dst, size_t n, int es, void *state, hipStream_t st,
                   unsigned spins) {
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
                                                                                  spins);
      break;
    }
    case 2: {
      const size_t npart = (units + d1p_units<2>() - 1) / d1p_units<2>();
      static const unsigned cap = resident_grid(k_delta_dec1p<2>, ~(size_t)0 >> 1);
      k_delta_dec1p<2><<<(unsigned)(npart < cap ? npart : cap), MC_BLOCK, 0, st>>>(s, d, units, ws, npart,
                                                                                  spins);
      break;
    }
    default: {
      const size_t npart = (units + d1p_units<4>() - 1) / d1p_units<4>();
      static const unsigned cap = resident_grid(k_delta_dec1p<4>, ~(size_t)0 >> 1);
      k_delta_dec1p<4><<<(unsigned)(npart < cap ? npart : cap), MC_BLOCK, 0, st>>>(s, d, units, ws, npart,
                                                                                  spins);
      break;
    }
  }
  return mc_last_launch();
}

size_t mc_c4_dec1p_state_bytes(size_t n, int astype) {
  const size_t E = (astype == MC_I2 || astype == MC_U2) ? 32768 : 16384;
  return mc_lb_ws_bytes((n + E - 1) / E);
}

// the fused FSO <- Delta <- Shuffle decode (c4_ok shapes), single pass;
// `state` = mc_c4_dec1p_state_bytes(n, astype) zeroed bytes
int mc_c4_dec1p(const void *src, void *dst, size_t n, int astype, int dtype, double scale, double offset,
                void *state, hipStream_t st, unsigned spins) {
  if (!c4_ok(src, dst, n, dtype, astype) || (uintptr_t)state % 16) return MC_EINVAL;
  const C4Params p = c4_decode_params(n, scale, offset);
  const uint8_t *s = static_cast<const uint8_t *>(src);
  uint8_t *d = static_cast<uint8_t *>(dst);
  uint32_t *ws = static_cast<uint32_t *>(state);
  MC_C4_DISPATCH(launch_c4_dec1p, s, d, ws, p, spins, st);
  return mc_last_launch();
}
