// Latency of dependent wave-scan steps: 64-bit vs 32-bit __shfl_up chains and
// DPP row operations.  Tuning tool only.
#include <cstdio>
#include "../numcodecs_amd/csrc/mc_scan.h"

template <typename T, int N>
__global__ __launch_bounds__(64) void k_chain(T *p) {
  T v = p[threadIdx.x];
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const T o = __shfl_up(v, off, 64);
      if ((threadIdx.x & 63) >= off) v += o;
    }
  }
  p[threadIdx.x] = v;
}

template <int N>
__global__ __launch_bounds__(64) void k_chain_lib(uint64_t *p) {
  uint64_t v = p[threadIdx.x];
  for (int i = 0; i < N; ++i) v = mc_wave_incl_scan<false>(v);
  p[threadIdx.x] = v;
}

template <typename K>
float time_it(K k, uint64_t *d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<<<1, 64>>>(reinterpret_cast<decltype(d)>(d));
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 20; ++r) k<<<1, 64>>>(d);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return 1000 * ms / 20;
}

int main() {
  uint64_t *d;
  hipMalloc(&d, 4096);
  hipMemset(d, 0, 4096);
  printf("{\"u64_chain1\": %.2f, \"u64_chain16\": %.2f, \"u64_chain64\": %.2f, ",
         time_it(k_chain<uint64_t, 1>, d), time_it(k_chain<uint64_t, 16>, d), time_it(k_chain<uint64_t, 64>, d));
  printf("\"lib_chain16\": %.2f, \"lib_chain64\": %.2f, ", time_it(k_chain_lib<16>, d), time_it(k_chain_lib<64>, d));
  uint32_t *d32 = reinterpret_cast<uint32_t *>(d);
  auto t32 = [&](auto k) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    k<<<1, 64>>>(d32); hipDeviceSynchronize();
    hipEventRecord(a); for (int r = 0; r < 20; ++r) k<<<1, 64>>>(d32); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); return 1000 * ms / 20;
  };
  printf("\"u32_chain16\": %.2f, \"u32_chain64\": %.2f}\n", t32(k_chain<uint32_t, 16>), t32(k_chain<uint32_t, 64>));
  return 0;
}
