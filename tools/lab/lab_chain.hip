// lab_chain.hip -- LAB ONLY (libmcodec_lab.so): the float Delta decode's
// serial chain (numpy's cumsum order, one dependent add per element) fed
// from LDS by one lane, in several instruction schedules, to find where the
// chain lane's time goes (tools/probe_chain.py).  One wave; lane 0 runs the
// chain over an LDS buffer of `n` floats `reps` times, in place.
//   kind 0  register-only chain (no LDS traffic): the dependent-add floor
//   kind 1  the product's schedule (mc_fspec.h fsw_chain: 32-value groups,
//           two register sets alternating, all reads of the next group
//           issued before the current group's adds)
//   kind 2  strict interleave: every 4 adds of the current group are
//           followed by one ds_write_b128 of the previous group's results
//           and one ds_read_b128 of the next group (sched_group_barrier)
//   kind 3  reads only (the results are not written back)
//   kind 4  DPP-fed adds: lanes 0-15 load 64 values with one ds_read_b128
//           each, lane 0 adds them through v_add_f32 with a row_shl source
//           (no per-element move), results written by lane 0 as 16-B stores
//   kinds 5-10  NS register sets of G values rotating (k_lab_chain_rot):
//           group t's adds, the store of group t-1 (computed a whole group
//           earlier, so the store never waits on its data and nothing
//           overwrites its registers soon after), the load of group t+NS-2
//           into the set stored one step ago.  ORD 0 = adds first, ORD 1 =
//           store + load first.  5: G16 NS4, 6: G16 NS8, 7: G32 NS4,
//           8: G16 NS4 ORD1, 9: G8 NS8, 10: G16 NS8 ORD1
//   kinds 11-15  SGPR-fed chain (k_lab_chain_sgpr): the inputs come from
//           global memory through scalar loads (constant address space), so
//           the adds read SGPR operands and no input passes through VGPRs;
//           the chain runs in every lane (uniform).  11: no result stores,
//           12: lane 0 writes the results to LDS (ds_write_b128), 13: lane 0
//           writes them to global memory (16-B stores), 14: kind 1's LDS-fed
//           chain with global result stores, 15: SGPR-fed, results gathered
//           into lane k of a VGPR (v_cndmask per element) and written as one
//           wave-wide 4-B store per 64 elements
//   kinds 16-18  kind 13 run redundantly by WAVES waves (one per SIMD): every
//           wave computes the whole chain, wave w stores only the 32-value
//           groups g with g % WAVES == w, so each wave's store cost per
//           element drops by WAVES.  16: 4 waves, 17: 2 waves, 18: 8 waves
//   kinds 19-21  kind 13 variants: 19 stores only every 16th group (is it
//           the stores or the distinct result registers?), 20 stores each
//           value with its own 4-B store, 21 stores a group only after the
//           next group's adds (two result sets alternate)
//   kinds 22-23  the chain values are the same in every lane, so every lane
//           stores them (same addresses, no lane-0 branch that lets the
//           compiler sink the adds past the stores): 22 = kind 21's lagging
//           stores, 23 = kind 13's
//   kinds 24-25  kind 1 / kind 14 (LDS-fed) run by all 64 lanes of the wave
//           (uniform chain, broadcast LDS reads, same-address stores): 24
//           writes the results back to LDS, 25 to global memory
#include "mc_scan.h"

namespace {

constexpr int CG = 32;  // values per group

template <int CTRL>
MC_DEV float lab_shl(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}

// acc + (value of lane + K of `v`), K = 1..15, as one DPP-sourced add
template <int K>
MC_DEV float lab_add_shl(float acc, float v) {
  if constexpr (K == 0) return acc + v;
  else return acc + lab_shl<0x100 + K>(v);
}

template <int K>
MC_DEV void lab_dpp_group(float &acc, const float (&v)[4], float (&r)[64]) {
  if constexpr (K < 16) {
    acc = lab_add_shl<K>(acc, v[0]);
    r[4 * K] = acc;
    acc = lab_add_shl<K>(acc, v[1]);
    r[4 * K + 1] = acc;
    acc = lab_add_shl<K>(acc, v[2]);
    r[4 * K + 2] = acc;
    acc = lab_add_shl<K>(acc, v[3]);
    r[4 * K + 3] = acc;
    lab_dpp_group<K + 1>(acc, v, r);
  }
}

template <int KIND>
__global__ __launch_bounds__(64) void k_lab_chain(const float *__restrict__ init, float *__restrict__ out,
                                                 long long *__restrict__ cyc, int n, int reps) {
  __shared__ __attribute__((aligned(16))) float p[8192 + 4 * CG];
  for (int i = threadIdx.x; i < n + 4 * CG; i += 64) p[i] = init[i % 64];
  __syncthreads();
  float acc = 0.0f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (KIND == 0) {
    if (threadIdx.x == 0) {
      float v[16];
      for (int k = 0; k < 16; ++k) v[k] = p[k];
      for (int r = 0; r < reps; ++r)
        for (int j = 0; j < n; j += 16) {
#pragma unroll
          for (int k = 0; k < 16; ++k) acc = acc + v[k];
          v[j & 15] = acc;
        }
    }
  } else if constexpr (KIND == 1 || KIND == 3 || KIND == 24) {
    if (KIND == 24 || threadIdx.x == 0) {
      for (int r = 0; r < reps; ++r) {
        float ga[CG], gb[CG];
        ser_ld<float, CG>(p, ga);
        for (int j = 0; j + 2 * CG <= n; j += 2 * CG) {
          ser_ld<float, CG>(p + j + CG, gb);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < CG; ++k) {
            acc = acc + ga[k];
            ga[k] = acc;
          }
          if constexpr (KIND != 3) ser_st<float, CG>(p + j, ga);
          ser_ld<float, CG>(p + j + 2 * CG, ga);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < CG; ++k) {
            acc = acc + gb[k];
            gb[k] = acc;
          }
          if constexpr (KIND != 3) ser_st<float, CG>(p + j + CG, gb);
          else acc += gb[0] * 0.0f;
        }
      }
    }
  } else if constexpr (KIND == 2) {
    if (threadIdx.x == 0) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      for (int r = 0; r < reps; ++r) {
        f4v ga[CG / 4], gb[CG / 4];
#pragma unroll
        for (int k = 0; k < CG / 4; ++k) ga[k] = reinterpret_cast<const f4v *>(p)[k];
#pragma unroll
        for (int k = 0; k < CG / 4; ++k) gb[k] = reinterpret_cast<const f4v *>(p + CG)[k];
        for (int j = 0; j + 2 * CG <= n; j += 2 * CG) {
          // adds on ga (group j); write gb? no: gb is the next group (loaded);
          // results of ga go back in place after its adds, interleaved with
          // the loads of group j + 2G into ga's slots as they free up
#pragma unroll
          for (int k = 0; k < CG / 4; ++k) {
            float a0 = ga[k].x, a1 = ga[k].y, a2 = ga[k].z, a3 = ga[k].w;
            acc = acc + a0; a0 = acc;
            acc = acc + a1; a1 = acc;
            acc = acc + a2; a2 = acc;
            acc = acc + a3; a3 = acc;
            reinterpret_cast<f4v *>(p + j)[k] = f4v{a0, a1, a2, a3};
            ga[k] = reinterpret_cast<const f4v *>(p + j + 2 * CG)[k];
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
#pragma unroll
          for (int k = 0; k < CG / 4; ++k) {
            float a0 = gb[k].x, a1 = gb[k].y, a2 = gb[k].z, a3 = gb[k].w;
            acc = acc + a0; a0 = acc;
            acc = acc + a1; a1 = acc;
            acc = acc + a2; a2 = acc;
            acc = acc + a3; a3 = acc;
            reinterpret_cast<f4v *>(p + j + CG)[k] = f4v{a0, a1, a2, a3};
            gb[k] = reinterpret_cast<const f4v *>(p + j + 3 * CG)[k];
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
        }
      }
    }
  } else {  // KIND 4: DPP-fed adds, lanes 0-15 hold 64 values
    typedef float f4v __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x;
    for (int r = 0; r < reps; ++r) {
      for (int j = 0; j + 64 <= n; j += 64) {
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (lane < 16) {
          const f4v x = reinterpret_cast<const f4v *>(p + j)[lane];
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        }
        // element 4K + c sits in v[c] of lane K: lane 0 adds it with row_shl:K
        float res[64];
        lab_dpp_group<0>(acc, v, res);
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < 16; ++k)
            reinterpret_cast<f4v *>(p + j)[k] = f4v{res[4 * k], res[4 * k + 1], res[4 * k + 2], res[4 * k + 3]};
        }
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = acc + p[7];
    cyc[0] = t1 - t0;
  }
}

template <int G, int NS, int ORD>
__global__ __launch_bounds__(64) void k_lab_chain_rot(const float *__restrict__ init, float *__restrict__ out,
                                                     long long *__restrict__ cyc, int n, int reps) {
  __shared__ __attribute__((aligned(16))) float p[8192 + 4 * CG];
  for (int i = threadIdx.x; i < n + 4 * CG; i += 64) p[i] = init[i % 64];
  __syncthreads();
  float acc = 0.0f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    constexpr int P = NS - 2;  // prefetch distance in groups
    float s[NS][G];
    const int mask = n - 1;    // n is a power of two
#pragma unroll
    for (int u = 0; u < P; ++u) ser_ld<float, G>(p + u * G, s[u]);
    int base = 0;
    const int steps = (n / G) * reps;
    for (int t = 0; t < steps; t += NS) {
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        constexpr int dummy = 0;
        (void)dummy;
        float(&cur)[G] = s[u];
        float(&prev)[G] = s[(u + NS - 1) % NS];
        float(&nxt)[G] = s[(u + P) % NS];
        const int pa = (base - G) & mask, la = (base + P * G) & mask;
        if constexpr (ORD == 1) {
          if (t + u > 0) ser_st<float, G>(p + pa, prev);
          ser_ld<float, G>(p + la, nxt);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
          acc = acc + cur[k];
          cur[k] = acc;
        }
        if constexpr (ORD == 0) {
          __builtin_amdgcn_sched_barrier(0);
          if (t + u > 0) ser_st<float, G>(p + pa, prev);
          ser_ld<float, G>(p + la, nxt);
        }
        __builtin_amdgcn_sched_barrier(0);
        base = (base + G) & mask;
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = acc + p[7];
    cyc[0] = t1 - t0;
  }
}

typedef const __attribute__((address_space(4))) float *cfp;

template <int KIND, int WAVES = 1>
__global__ __launch_bounds__(64 * WAVES) void k_lab_chain_sgpr(const float *__restrict__ init, float *__restrict__ out,
                                                      long long *__restrict__ cyc, int n, int reps,
                                                      const float *__restrict__ gin, float *__restrict__ gout) {
  __shared__ __attribute__((aligned(16))) float p[8192 + 4 * CG];
  for (int i = threadIdx.x; i < n + 4 * CG; i += 64 * WAVES) p[i] = init[i % 64];
  __syncthreads();
  typedef float f4v __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float acc = 0.0f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (KIND == 14 || KIND == 25) {
    if (KIND == 25 || lane == 0) {
      for (int r = 0; r < reps; ++r) {
        float ga[CG], gb[CG];
        ser_ld<float, CG>(p, ga);
        for (int j = 0; j + 2 * CG <= n; j += 2 * CG) {
          ser_ld<float, CG>(p + j + CG, gb);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < CG; ++k) {
            acc = acc + ga[k];
            ga[k] = acc;
          }
          ser_st<float, CG>(gout + j, ga);
          ser_ld<float, CG>(p + j + 2 * CG, ga);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < CG; ++k) {
            acc = acc + gb[k];
            gb[k] = acc;
          }
          ser_st<float, CG>(gout + j + CG, gb);
        }
      }
    }
  } else if constexpr (KIND == 21 || KIND == 22) {
    cfp src = (cfp)gin;
    constexpr int SG = 32;
    auto sld = [&](int at, float (&g)[SG]) {
#pragma unroll
      for (int k = 0; k < SG; ++k) g[k] = src[at + k];
    };
    auto st = [&](int at, const float (&r)[SG]) {
      if (KIND == 22 || lane == 0) {
#pragma unroll
        for (int k = 0; k < SG / 4; ++k)
          reinterpret_cast<f4v *>(gout + at)[k] = f4v{r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]};
      }
    };
    if constexpr (KIND == 21) {
      for (int r = 0; r < reps; ++r) {
        float ga[SG], gb[SG], ra[SG], rb[SG];
        sld(0, ga);
#pragma unroll
        for (int k = 0; k < SG; ++k) rb[k] = 0.0f;
        for (int j = 0; j < n; j += 2 * SG) {
          const int jj = __builtin_amdgcn_readfirstlane(j);
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_sched_barrier(0);
          sld(jj + SG, gb);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < SG; ++k) {
            acc = acc + ga[k];
            ra[k] = acc;
          }
          __builtin_amdgcn_sched_barrier(0);
          st((jj - SG) & (n - 1), rb);  // the previous group, computed a group ago
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_sched_barrier(0);
          sld((jj + 2 * SG) & (n - 1), ga);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < SG; ++k) {
            acc = acc + gb[k];
            rb[k] = acc;
          }
          __builtin_amdgcn_sched_barrier(0);
          st(jj, ra);
          __builtin_amdgcn_sched_barrier(0);
        }
        // the last group's results are still pending (round 4 left them out:
        // the "one group late" store of the first group wrote zeros there)
        st(n - SG, rb);
      }
    } else {
      // 4 result sets: group t writes S[t % 4], the stores of S[(t-1) % 4]
      // follow its adds, and S[(t-2) % 4] is kept alive (empty asm use) until
      // after them, so no add ever writes a register a store issued less
      // than a whole group earlier may still be reading
      for (int r = 0; r < reps; ++r) {
        float G[2][SG], S[4][SG];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int k = 0; k < SG; ++k) S[u][k] = 0.0f;
        sld(0, G[0]);
        for (int j = 0; j < n; j += 4 * SG) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int jj = __builtin_amdgcn_readfirstlane(j + u * SG);
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_sched_barrier(0);
            sld((jj + SG) & (n - 1), G[(u + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < SG; ++k) {
              acc = acc + G[u & 1][k];
              S[u][k] = acc;
            }
            __builtin_amdgcn_sched_barrier(0);
            st((jj - SG) & (n - 1), S[(u + 3) & 3]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < SG; ++k) asm volatile("" ::"v"(S[(u + 2) & 3][k]));
          }
        }
        st(n - SG, S[3]);  // the last group (stored one group late, after the loop)
      }
    }
  } else {
    cfp src = (cfp)gin;
    constexpr int SG = 32;  // SGPR group: two alternate, the next one's scalar loads in flight
    auto sld = [&](int at, float (&g)[SG]) {
#pragma unroll
      for (int k = 0; k < SG; ++k) g[k] = src[at + k];
    };
    auto group = [&](int j, const float (&g)[SG], float &gat, int k0) {
      float res[SG];
#pragma unroll
      for (int k = 0; k < SG; ++k) {
        acc = acc + g[k];
        if constexpr (KIND == 15) gat = lane == k0 + k ? acc : gat;
        else res[k] = acc;
      }
      if constexpr (KIND == 12) {
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < SG / 4; ++k)
            reinterpret_cast<f4v *>(p + j)[k] = f4v{res[4 * k], res[4 * k + 1], res[4 * k + 2], res[4 * k + 3]};
        }
      } else if constexpr (KIND == 19) {
        if (lane == 0 && (j & (16 * SG - 1)) == 0) {
#pragma unroll
          for (int k = 0; k < SG / 4; ++k)
            reinterpret_cast<f4v *>(gout + j)[k] = f4v{res[4 * k], res[4 * k + 1], res[4 * k + 2], res[4 * k + 3]};
        }
      } else if constexpr (KIND == 20) {
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < SG; ++k) gout[j + k] = res[k];
        }
      } else if constexpr (KIND == 23) {
#pragma unroll
        for (int k = 0; k < SG / 4; ++k)
          reinterpret_cast<f4v *>(gout + j)[k] = f4v{res[4 * k], res[4 * k + 1], res[4 * k + 2], res[4 * k + 3]};
      } else if constexpr (KIND == 13) {
        if (lane == 0 && (WAVES == 1 || ((j / SG) % WAVES) == wave)) {
#pragma unroll
          for (int k = 0; k < SG / 4; ++k)
            reinterpret_cast<f4v *>(gout + j)[k] = f4v{res[4 * k], res[4 * k + 1], res[4 * k + 2], res[4 * k + 3]};
        }
      } else {
        (void)res;
      }
    };
    for (int r = 0; r < reps; ++r) {
      float ga[SG], gb[SG];
      sld(0, ga);
      for (int j = 0; j < n; j += 2 * SG) {
        const int jj = __builtin_amdgcn_readfirstlane(j);
        float gat = 0.0f;
        // SMEM returns out of order, so any wait is lgkmcnt(0): wait for the
        // current group first, then issue the next group's loads
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        sld(jj + SG, gb);
        __builtin_amdgcn_sched_barrier(0);
        group(jj, ga, gat, 0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        sld((jj + 2 * SG) & (n - 1), ga);
        __builtin_amdgcn_sched_barrier(0);
        group(jj + SG, gb, gat, SG);
        if constexpr (KIND == 15) gout[jj + lane] = gat;
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = acc + p[7];
    cyc[0] = t1 - t0;
  }
}

// ---------------------------------------------------------------------------
// f64 chains (round 5): the dependent v_add_f64 floor and the SGPR-fed /
// LDS-fed schedules of the product's f8 walker, one wave
//   kind 40  register-only chain
//   kind 41  SGPR-fed (s_load of the inputs), no result stores
//   kind 42  SGPR-fed, every lane stores the (uniform) results, 16-B stores
//   kind 43  LDS-fed, lane 0 stores to global (the product's f8 fsw_chain)
//   kind 44  SGPR-fed, lane 0 stores to global
// ---------------------------------------------------------------------------
typedef const __attribute__((address_space(4))) double *cdp;

template <int KIND>
__global__ __launch_bounds__(64) void k_lab_chain64(const double *__restrict__ init, double *__restrict__ out,
                                                   long long *__restrict__ cyc, int n, int reps,
                                                   const double *__restrict__ gin, double *__restrict__ gout) {
  constexpr int SG = 16;  // values per group
  __shared__ __attribute__((aligned(16))) double p[4096 + 4 * SG];
  for (int i = threadIdx.x; i < n + 4 * SG; i += 64) p[i] = i < n ? gin[i] : init[i % 64];
  __syncthreads();
  typedef double d2v __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (KIND == 40) {
    if (lane == 0) {
      double v[16];
      for (int k = 0; k < 16; ++k) v[k] = p[k];
      for (int r = 0; r < reps; ++r)
        for (int j = 0; j < n; j += 16) {
#pragma unroll
          for (int k = 0; k < 16; ++k) acc = acc + v[k];
          v[j & 15] = acc;
        }
    }
  } else if constexpr (KIND == 43) {
    if (lane == 0) {
      for (int r = 0; r < reps; ++r) {
        double ga[SG], gb[SG];
        ser_ld<double, SG>(p, ga);
        for (int j = 0; j + 2 * SG <= n; j += 2 * SG) {
          ser_ld<double, SG>(p + j + SG, gb);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < SG; ++k) {
            acc = acc + ga[k];
            ga[k] = acc;
          }
          ser_st<double, SG>(gout + j, ga);
          ser_ld<double, SG>(p + j + 2 * SG, ga);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < SG; ++k) {
            acc = acc + gb[k];
            gb[k] = acc;
          }
          ser_st<double, SG>(gout + j + SG, gb);
        }
      }
    }
  } else {
    cdp src = (cdp)gin;
    auto sld = [&](int at, double (&g)[SG]) {
#pragma unroll
      for (int k = 0; k < SG; ++k) g[k] = src[at + k];
    };
    auto group = [&](int j, const double (&g)[SG]) {
      double res[SG];
#pragma unroll
      for (int k = 0; k < SG; ++k) {
        acc = acc + g[k];
        res[k] = acc;
      }
      if constexpr (KIND == 42) {
#pragma unroll
        for (int k = 0; k < SG / 2; ++k) reinterpret_cast<d2v *>(gout + j)[k] = d2v{res[2 * k], res[2 * k + 1]};
      } else if constexpr (KIND == 44) {
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < SG / 2; ++k) reinterpret_cast<d2v *>(gout + j)[k] = d2v{res[2 * k], res[2 * k + 1]};
        }
      } else {
        (void)res;
      }
    };
    for (int r = 0; r < reps; ++r) {
      double ga[SG], gb[SG];
      sld(0, ga);
      for (int j = 0; j < n; j += 2 * SG) {
        const int jj = __builtin_amdgcn_readfirstlane(j);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        sld(jj + SG, gb);
        __builtin_amdgcn_sched_barrier(0);
        group(jj, ga);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        sld((jj + 2 * SG) & (n - 1), ga);
        __builtin_amdgcn_sched_barrier(0);
        group(jj + SG, gb);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = acc + p[7];
    cyc[0] = t1 - t0;
  }
}

// ---------------------------------------------------------------------------
// LAB: the chain fed from SGPRs (round 5, lab kinds 23 / 42,
// profiles/r05/probe_chain_r5.jsonl): every lane of the calling wave runs the
// same dependent adds, the operands coming from scalar loads straight out of
// global memory (s_load_dwordxN: no VGPR or LDS staging of the inputs, the
// adds read SGPRs), and every lane stores the (uniform) results as 16-B
// vectors to the same addresses -- no lane-0 branch for the compiler to sink
// the adds past.  Measured per element: f32 9.4 ticks against 11.0 for the
// LDS-fed lane-0 chain, f64 14.9 against 18.7.  Two scalar groups of SG
// values alternate, the next group's loads issued after the current group's
// have landed (scalar loads return out of order: any wait is lgkmcnt(0)).
// `in` / `out`: element pointers (uniform), `out` 16-B aligned; cnt elements.
// Only for f4 / f8 with astype == dtype, little-endian.
// ---------------------------------------------------------------------------
// `prog` (LDS, may be null): the chain publishes how many of the cnt
// elements it has consumed, for ser_prefetch in another wave.
template <typename T, int SG = sizeof(T) == 8 ? 16 : 32>  // SG: values per scalar group
MC_DEV T ser_chain_sgpr(const T *in, T *out, size_t cnt, T acc, volatile size_t *prog = nullptr) {
  constexpr int W = 16 / (int)sizeof(T);
  typedef const __attribute__((address_space(4))) T *cp;
  typedef T vec __attribute__((ext_vector_type(W)));
  // stores through a global (not flat) pointer: flat stores count in
  // lgkmcnt too, so the lgkmcnt(0) waits for the scalar loads would also
  // wait for every store to land
  typedef __attribute__((address_space(1))) T *gp;
  typedef __attribute__((address_space(1))) vec *gvp;
  in = mc_uniform_ptr(in);
  const gp dstp = (gp)mc_uniform_ptr(out);
  const cp src = (cp)in;
  size_t j = 0;
  // head: up to the first 16-B aligned output element
  for (; j < cnt && (((uintptr_t)(out + j)) & 15); ++j) {
    acc = acc + src[j];
    dstp[j] = acc;
  }
  auto sld = [&](size_t at, T(&g)[SG]) {
    const cp q = mc_uniform_ptr(src + at);
#pragma unroll
    for (int k = 0; k < SG; ++k) g[k] = q[k];
  };
  auto group = [&](size_t at, const T(&g)[SG]) {
    T res[SG];
#pragma unroll
    for (int k = 0; k < SG; ++k) {
      acc = acc + g[k];
      res[k] = acc;
    }
    const gvp o = (gvp)(dstp + at);
#pragma unroll
    for (int k = 0; k < SG / W; ++k) {
      vec v;
#pragma unroll
      for (int e = 0; e < W; ++e) v[e] = res[W * k + e];
      o[k] = v;
    }
  };
  if (j + 2 * SG <= cnt) {
    T ga[SG], gb[SG];
    sld(j, ga);
    for (; j + 2 * SG <= cnt; j += 2 * SG) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): group ga has landed
      __builtin_amdgcn_sched_barrier(0);
      sld(j + SG, gb);
      if (prog) *(volatile __attribute__((address_space(3))) size_t *)prog = j;
      __builtin_amdgcn_sched_barrier(0);
      group(j, ga);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      if (j + 3 * SG <= cnt) sld(j + 2 * SG, ga);  // never past the input
      __builtin_amdgcn_sched_barrier(0);
      group(j + SG, gb);
    }
  }
  for (; j < cnt; ++j) {
    acc = acc + src[j];
    dstp[j] = acc;
  }
  return acc;
}

// The scalar loads above see HBM's miss latency (~900 cycles) once per
// group, longer than a group's adds (32 x ~9 cycles): a 256 MiB f4 chain ran
// at 720 ms, against 360 ms for the LDS-fed one.  Scalar returns come back
// out of order, so the chain cannot keep more than one group in flight; one
// other wave of the workgroup instead keeps its input ahead of it in the
// caches: vector loads (one dword per 128-B line) SER_PF_L2 bytes past the
// chain's published position pull the lines into L2, and scalar loads (one
// dword per 64-B line) SER_PF_K bytes past it pull them into the CU's scalar
// cache, where the chain's own scalar loads then hit.  The wave sleeps while
// it is that far ahead, never blocks the chain, and ends once the whole input
// is requested (the chain's last published position is within 2 groups of
// the end, so both windows reach it) or the chain signals its end (~0).
// ---------------------------------------------------------------------------
constexpr size_t SER_PF_L2 = 32768;
constexpr size_t SER_PF_K = 0;  // the scalar-cache window: off (see below)

MC_DEV void ser_prefetch(const void *in, size_t bytes, size_t es, volatile size_t *prog,
                         size_t l2_ahead = SER_PF_L2, size_t k_ahead = SER_PF_K) {
  typedef const __attribute__((address_space(4))) uint32_t *cp;
  const int lane = threadIdx.x & 63;
  const uint8_t *base = mc_uniform_ptr(reinterpret_cast<const uint8_t *>((uintptr_t)in & ~(uintptr_t)127));
  const size_t span = bytes + ((uintptr_t)in & 127);
  size_t pf2 = 0, pfk = 0;
  uint32_t seen = 0;  // keeps the loads (a value no one reads)
  if (k_ahead == 0) pfk = span;
  while (pf2 < span || pfk < span) {
    const size_t at = *prog;
    if (at == ~(size_t)0) break;  // the chain has finished (k_lab_stream)
    const size_t pos = at * es;
    const size_t t2 = pos + l2_ahead < span ? pos + l2_ahead : span;
    const size_t tk = pos + k_ahead < span ? pos + k_ahead : span;
    bool idle = true;
    if (pf2 < t2) {
      const size_t o = pf2 + (size_t)lane * 128;
      if (o < span) seen ^= *reinterpret_cast<const uint32_t *>(base + o);
      pf2 += 64 * 128;
      idle = false;
    }
    if (pfk < tk) {
      const cp q = (cp)(base + pfk);
      uint32_t k = 0;
#pragma unroll
      for (int l = 0; l < 16; ++l)
        if (pfk + 64 * l < span) k ^= q[16 * l];
      seen ^= k;
      pfk += 16 * 64;
      idle = false;
    }
    if (idle) __builtin_amdgcn_s_sleep(2);
  }
  [[maybe_unused]] __shared__ uint32_t sink;
  if (seen == 0x9E3779B9u) sink = seen;
}

// ---------------------------------------------------------------------------
// Streaming chains (round 5): the lab's ser_chain_sgpr above (kinds 0 f32,
// 1 f64) or ser_chain_vbc (kinds 2 f32, 3 f64; `ka` = its depth D) over a
// large buffer (HBM, not cache-resident like kinds 11-25), wave 1 running
// ser_prefetch with the given windows (pf = 0: no prefetch wave).  Finds the
// group size and prefetch distances that hide the loads' latency.
// ---------------------------------------------------------------------------
template <typename T, int SG, int VD = 0>
__global__ __launch_bounds__(128) void k_lab_stream(const T *__restrict__ in, T *__restrict__ out, size_t n,
                                                    size_t l2a, size_t ka, int pf, long long *__restrict__ cyc) {
  __shared__ size_t prog;
  if (threadIdx.x == 0) prog = 0;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < 64) {
    T acc = in[0];
    if (threadIdx.x == 0) out[0] = acc;
    if constexpr (VD > 0) acc = ser_chain_vbc<T, SG, VD>(in + 1, out + 1, n - 1, acc);
    else acc = ser_chain_sgpr<T, SG>(in + 1, out + 1, n - 1, acc, &prog);
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      cyc[0] = t1 - t0;
      *(volatile size_t *)&prog = ~(size_t)0;  // the prefetch wave's exit, whatever it has requested
    }
  } else if (pf) {
    ser_prefetch(in + 1, (n - 1) * sizeof(T), sizeof(T), &prog, l2a, ka);
  }
}

}  // namespace

extern "C" int mc_lab_chain64(const double *init, double *out, long long *cyc, int n, int reps, int kind,
                              const double *gin, double *gout, mc_stream_t stream) {
  if (n <= 0 || n > 4096 || (n & (n - 1)) || n < 64 || reps <= 0) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 40: k_lab_chain64<40><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 41: k_lab_chain64<41><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 42: k_lab_chain64<42><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 43: k_lab_chain64<43><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 44: k_lab_chain64<44><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    default: return MC_EINVAL;
  }
  return mc_last_launch();
}

extern "C" int mc_lab_chain(const float *init, float *out, long long *cyc, int n, int reps, int kind,
                            mc_stream_t stream) {
  if (n <= 0 || n > 8192 || n % 128 || reps <= 0) return MC_EINVAL;
  if (kind >= 5 && (n & (n - 1))) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 0: k_lab_chain<0><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 1: k_lab_chain<1><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 2: k_lab_chain<2><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 3: k_lab_chain<3><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 4: k_lab_chain<4><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 24: k_lab_chain<24><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 5: k_lab_chain_rot<16, 4, 0><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 6: k_lab_chain_rot<16, 8, 0><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 7: k_lab_chain_rot<32, 4, 0><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 8: k_lab_chain_rot<16, 4, 1><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 9: k_lab_chain_rot<8, 8, 0><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 10: k_lab_chain_rot<16, 8, 1><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    default: return MC_EINVAL;
  }
  return mc_last_launch();
}

// kinds 11-15: gin = n input floats in global memory, gout = n output floats
extern "C" int mc_lab_chain_g(const float *init, float *out, long long *cyc, int n, int reps, int kind,
                              const float *gin, float *gout, mc_stream_t stream) {
  if (n <= 0 || n > 8192 || n % 128 || (n & (n - 1)) || reps <= 0) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 11: k_lab_chain_sgpr<11><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 12: k_lab_chain_sgpr<12><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 13: k_lab_chain_sgpr<13><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 14: k_lab_chain_sgpr<14><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 15: k_lab_chain_sgpr<15><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 16: k_lab_chain_sgpr<13, 4><<<1, 256, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 17: k_lab_chain_sgpr<13, 2><<<1, 128, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 18: k_lab_chain_sgpr<13, 8><<<1, 512, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 19: k_lab_chain_sgpr<19><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 20: k_lab_chain_sgpr<20><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 21: k_lab_chain_sgpr<21><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 22: k_lab_chain_sgpr<22><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 23: k_lab_chain_sgpr<23><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    case 25: k_lab_chain_sgpr<25><<<1, 64, 0, st>>>(init, out, cyc, n, reps, gin, gout); break;
    default: return MC_EINVAL;
  }
  return mc_last_launch();
}

// in / out: n elements (kind 0 f32, kind 1 f64); sg selects the group size
extern "C" int mc_lab_stream(const void *in, void *out, size_t n, int kind, int sg, size_t l2a, size_t ka, int pf,
                             long long *cyc, mc_stream_t stream) {
  if (n < 2) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const float *fi = (const float *)in;
  float *fo = (float *)out;
  const double *di = (const double *)in;
  double *dout = (double *)out;
#define LS(T, G, I, O) k_lab_stream<T, G><<<1, 128, 0, st>>>(I, O, n, l2a, ka, pf, cyc)
  if (kind == 0 && sg == 32) LS(float, 32, fi, fo);
  else if (kind == 0 && sg == 40) LS(float, 40, fi, fo);
  else if (kind == 0 && sg == 48) LS(float, 48, fi, fo);
  else if (kind == 0 && sg == 24) LS(float, 24, fi, fo);
  else if (kind == 1 && sg == 16) LS(double, 16, di, dout);
  else if (kind == 1 && sg == 20) LS(double, 20, di, dout);
  else if (kind == 1 && sg == 24) LS(double, 24, di, dout);
  else if (kind == 1 && sg == 12) LS(double, 12, di, dout);
  else if (kind >= 2) {
    const size_t d = ka;
    ka = 0;
    if ((uintptr_t)in % 16 != (uintptr_t)out % 16) return MC_EINVAL;
#define LV(T, G, V, I, O) k_lab_stream<T, G, V><<<1, 128, 0, st>>>(I, O, n, l2a, ka, pf, cyc)
    if (kind == 2 && sg == 32 && d == 6) LV(float, 32, 6, fi, fo);
    else if (kind == 2 && sg == 32 && d == 4) LV(float, 32, 4, fi, fo);
    else if (kind == 2 && sg == 24 && d == 8) LV(float, 24, 8, fi, fo);
    else if (kind == 2 && sg == 16 && d == 12) LV(float, 16, 12, fi, fo);
    else if (kind == 3 && sg == 16 && d == 6) LV(double, 16, 6, di, dout);
    else if (kind == 3 && sg == 12 && d == 8) LV(double, 12, 8, di, dout);
    else if (kind == 3 && sg == 8 && d == 12) LV(double, 8, 12, di, dout);
    else return MC_EINVAL;
#undef LV
#undef LV
  } else return MC_EINVAL;
#undef LS
  return mc_last_launch();
}
