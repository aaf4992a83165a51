// Host cost of one kernel launch on a stream, three ways: the triple-chevron
// launch, hipLaunchKernel with a prepared argument array, and
// hipModuleLaunchKernel on the hipFunction_t looked up once
// (hipGetFuncBySymbol).  Also the enqueue-to-completion time of one empty
// launch waited for by a spin on a pinned flag the kernel sets.
//
//   hipcc --offload-arch=gfx950 -O2 tools/probe_launch.hip -o tools/_build/probe_launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_touch(unsigned *flag, unsigned v, size_t n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  (void)n;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned *flag;
  CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent));
  *flag = 0;
  hipFunction_t fn;
  CK(hipGetFuncBySymbol(&fn, reinterpret_cast<const void *>(k_touch)));
  const int R = 2000;
  const dim3 grid(1024), block(256);
  size_t n = 1;
  unsigned v = 0;
  std::vector<double> t[3], done[3];
  for (int rep = 0; rep < 3 * R; ++rep) {
    const int way = rep % 3;
    ++v;
    void *args[] = {&flag, &v, &n};
    const double t0 = now_us();
    if (way == 0) {
      k_touch<<<grid, block, 0, st>>>(flag, v, n);
    } else if (way == 1) {
      CK(hipLaunchKernel(reinterpret_cast<const void *>(k_touch), grid, block, args, 0, st));
    } else {
      CK(hipModuleLaunchKernel(fn, grid.x, 1, 1, block.x, 1, 1, 0, st, args, nullptr));
    }
    const double t1 = now_us();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
    }
    const double t2 = now_us();
    CK(hipStreamSynchronize(st));
    if (rep >= 30) {
      t[way].push_back(t1 - t0);
      done[way].push_back(t2 - t0);
    }
  }
  const char *names[] = {"chevron", "hipLaunchKernel", "hipModuleLaunchKernel"};
  printf("{");
  for (int w = 0; w < 3; ++w) {
    std::sort(t[w].begin(), t[w].end());
    std::sort(done[w].begin(), done[w].end());
    printf("%s\"%s\": {\"launch_us_med\": %.2f, \"launch_us_p10\": %.2f, \"flag_seen_us_med\": %.2f}", w ? ", " : "",
           names[w], t[w][t[w].size() / 2], t[w][t[w].size() / 10], done[w][done[w].size() / 2]);
  }
  printf("}\n");
  CK(hipHostFree(flag));
  CK(hipStreamDestroy(st));
  return 0;
}
