// bwtest.hip -- HBM streaming calibration kernels (copy / read / write) used to
// find the load/store form that reaches the achievable HBM rate on MI355X.
// Not part of the product; built by tools/run_bwtest.py into tools/_build/.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ s, u32x4 *__restrict__ d,
                                              size_t nvec) {
  // each block moves U*256 u32x4 per iteration, grid-stride over tiles
  const size_t tiles = nvec / ((size_t)U * 256);
  for (size_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const size_t base = t * U * 256 + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT_LD) v[u] = __builtin_nontemporal_load(s + base + u * 256);
      else v[u] = s[base + u * 256];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT_ST) __builtin_nontemporal_store(v[u], d + base + u * 256);
      else d[base + u * 256] = v[u];
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const u32x4 *__restrict__ s, uint32_t *out, size_t nvec) {
  const size_t tiles = nvec / ((size_t)U * 256);
  uint32_t acc = 0;
  for (size_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const size_t base = t * U * 256 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      u32x4 v = s[base + u * 256];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int U, bool NT_ST>
__global__ __launch_bounds__(256) void k_write(u32x4 *__restrict__ d, size_t nvec) {
  const size_t tiles = nvec / ((size_t)U * 256);
  const u32x4 v = u32x4{threadIdx.x, blockIdx.x, 1u, 2u};
  for (size_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const size_t base = t * U * 256 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT_ST) __builtin_nontemporal_store(v, d + base + u * 256);
      else d[base + u * 256] = v;
    }
  }
}

extern "C" int bw_copy(const void *s, void *d, size_t nbytes, int variant, int grid, void *st) {
  const size_t nvec = nbytes / 16;
  hipStream_t stream = (hipStream_t)st;
  switch (variant) {
    case 0: k_copy<4, false, false><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 1: k_copy<4, false, true><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 2: k_copy<4, true, true><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 3: k_copy<1, false, false><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 4: k_copy<8, false, false><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 5: k_copy<8, false, true><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 6: k_copy<2, false, false><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 7: k_copy<4, true, false><<<grid, 256, 0, stream>>>((const u32x4 *)s, (u32x4 *)d, nvec); break;
    case 8: k_read<4><<<grid, 256, 0, stream>>>((const u32x4 *)s, (uint32_t *)d, nvec); break;
    case 9: k_write<4, false><<<grid, 256, 0, stream>>>((u32x4 *)d, nvec); break;
    case 10: k_write<4, true><<<grid, 256, 0, stream>>>((u32x4 *)d, nvec); break;
    default: return -22;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
