// Microbenchmark: cost of one dependent floating-point add chain on gfx950
// (the float Delta decode = np.cumsum is one such chain per chunk).
//   hipcc --offload-arch=gfx950 -O3 tools/chain_bench.hip -o tools/_build/chain_bench
// Prints cycles per add (s_memtime) and adds/s for: a register-only chain
// (f32, f64) with one lane active, and the same with many chains per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int LANES>
__global__ void k_chain(const T *x, T *out, long long *cyc, int iters) {
  T v[16];
  for (int k = 0; k < 16; ++k) v[k] = x[k + threadIdx.x % 4];
  T acc = x[0];
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < LANES) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = acc + v[k];
      v[i & 15] = acc;  // keep the loop body live
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x] = acc; cyc[blockIdx.x] = t1 - t0; }
}

template <typename T, int LANES>
static void run(const char *name, int blocks, int threads) {
  T *x, *out; long long *cyc;
  hipMalloc(&x, 64 * sizeof(T)); hipMemset(x, 0, 64 * sizeof(T));
  hipMalloc(&out, blocks * sizeof(T)); hipMalloc(&cyc, blocks * sizeof(long long));
  const int iters = 1 << 16;
  k_chain<T, LANES><<<blocks, threads>>>(x, out, cyc, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  k_chain<T, LANES><<<blocks, threads>>>(x, out, cyc, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c; hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  const double adds = 16.0 * iters;
  printf("{\"case\": \"%s\", \"blocks\": %d, \"threads\": %d, \"cycles_per_add\": %.2f, "
         "\"chain_Madds_per_s\": %.1f, \"total_Gadds_per_s\": %.2f}\n",
         name, blocks, threads, c / adds, adds / (ms * 1e-3) / 1e6,
         adds * blocks * (LANES < threads ? LANES : threads) / (ms * 1e-3) / 1e9);
  hipFree(x); hipFree(out); hipFree(cyc);
}

int main() {
  run<float, 1>("f32 one lane, one wave", 1, 64);
  run<double, 1>("f64 one lane, one wave", 1, 64);
  run<float, 1>("f32 one lane per wave, 1024 waves", 1024, 64);
  run<float, 1>("f32 one lane per wave, 4096 waves", 4096, 64);
  run<float, 64>("f32 64 lanes per wave, 4096 waves", 4096, 64);
  run<double, 1>("f64 one lane per wave, 4096 waves", 4096, 64);
  return 0;
}
