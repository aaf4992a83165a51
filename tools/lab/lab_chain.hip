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
  } else if constexpr (KIND == 1 || KIND == 3) {
    if (threadIdx.x == 0) {
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
          if constexpr (KIND == 1) ser_st<float, CG>(p + j, ga);
          ser_ld<float, CG>(p + j + 2 * CG, ga);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int k = 0; k < CG; ++k) {
            acc = acc + gb[k];
            gb[k] = acc;
          }
          if constexpr (KIND == 1) ser_st<float, CG>(p + j + CG, gb);
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

}  // namespace

extern "C" int mc_lab_chain(const float *init, float *out, long long *cyc, int n, int reps, int kind,
                            mc_stream_t stream) {
  if (n <= 0 || n > 8192 || n % 128 || reps <= 0) return MC_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  switch (kind) {
    case 0: k_lab_chain<0><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 1: k_lab_chain<1><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 2: k_lab_chain<2><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 3: k_lab_chain<3><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    case 4: k_lab_chain<4><<<1, 64, 0, st>>>(init, out, cyc, n, reps); break;
    default: return MC_EINVAL;
  }
  return mc_last_launch();
}
