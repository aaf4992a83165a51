// Microbenchmark of k_scan_sums (mc_scan.h) alone, sizes 16 .. 64K totals,
// and of an empty 1024-thread kernel, with HIP events.  Tuning tool only.
#include <cstdio>
#include <vector>
#include "../numcodecs_amd/csrc/mc_scan.h"

__global__ __launch_bounds__(1024) void k_empty(uint64_t *p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[0] = 1;
}

int main() {
  uint64_t *d;
  hipMalloc(&d, 65536 * 8);
  hipMemset(d, 0, 65536 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (size_t n : {16ul, 1024ul, 16384ul, 65536ul}) {
    std::vector<uint64_t> h(n, 1);
    hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice);
    k_scan_sums<false><<<1, 1024>>>(d, n);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, n * 8, hipMemcpyDeviceToHost);
    bool ok = true;
    for (size_t i = 0; i < n; ++i) ok &= h[i] == i;
    const int reps = 50;
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) k_scan_sums<false><<<1, 1024>>>(d, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"ntiles\": %zu, \"ok\": %d, \"us_per_launch\": %.2f}\n", n, ok, 1000 * ms / reps);
  }
  hipEventRecord(a);
  for (int r = 0; r < 50; ++r) k_empty<<<1, 1024>>>(d);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("{\"empty_1024\": %.2f}\n", 1000 * ms / 50);
  return 0;
}
