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
