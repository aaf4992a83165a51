// mc_misc.hip -- ABI version, status strings, device query.
#include "mc_common.h"

extern "C" {

int mc_abi_version(void) { return MC_ABI_VERSION; }

const char *mc_strerror(int status) {
  if (status == MC_OK) return "ok";
  if (status == MC_EINVAL) return "invalid argument";
  if (status == MC_ENOSPC) return "workspace too small";
  if (status == MC_EPROTO) return "the stream finished without publishing the verdict";
  if (status <= MC_EHIP_BASE) return hipGetErrorString((hipError_t)(MC_EHIP_BASE - status));
  return "unknown mcodec status";
}

int mc_stream_synchronize(mc_stream_t stream) {
  return mc_hip_status(hipStreamSynchronize((hipStream_t)stream));
}

void *mc_host_device_pointer(void *host) {
  void *d = nullptr;
  if (!host || hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return nullptr;
  return d;
}

void *mc_verdict_alloc(void) {
  void *p = nullptr;
  // fine-grained (coherent), mapped into every device's address space
  if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
    return nullptr;
  static_cast<uint32_t *>(p)[2] = 0;
  return p;
}

void mc_verdict_free(void *rec) {
  if (rec) (void)hipHostFree(rec);
}

int mc_verdict_wait(const uint32_t *rec, uint32_t seq, mc_stream_t stream) {
  if (!rec || !seq) return MC_EINVAL;
  for (unsigned i = 1;; ++i) {
    if (__atomic_load_n(&rec[2], __ATOMIC_ACQUIRE) == seq) return MC_OK;
    if ((i & 1023u) == 0) {  // every ~10-20 us: has the stream ended or failed?
      const hipError_t e = hipStreamQuery((hipStream_t)stream);
      if (e == hipSuccess)
        return __atomic_load_n(&rec[2], __ATOMIC_ACQUIRE) == seq ? MC_OK : MC_EPROTO;
      if (e != hipErrorNotReady) return mc_hip_status(e);
    }
    __builtin_ia32_pause();
  }
}

int mc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
