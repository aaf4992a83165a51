// mc_misc.hip -- ABI version, status strings, device query.
#include "mc_common.h"

extern "C" {

int mc_abi_version(void) { return MC_ABI_VERSION; }

const char *mc_strerror(int status) {
  if (status == MC_OK) return "ok";
  if (status == MC_EINVAL) return "invalid argument";
  if (status == MC_ENOSPC) return "workspace too small";
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

int mc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
