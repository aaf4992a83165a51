// mc_misc.hip -- ABI version, status strings, device query.
#include <time.h>

#include "mc_common.h"

// the measured defaults (mc_sched.h); nothing in the product changes them
mc_sched_t mc_sched = {
    /*copy_u*/ 4,         /*copy_grid*/ 0,     /*ck_k*/ 0,           /*ck_kcopy*/ 8,
    /*ck_grid*/ 0,        /*ck_grid_copy*/ 1024, /*f32_unroll*/ 0,    /*f32_ntld*/ 1,
    /*f32_fused_grid*/ 2048, /*f32_slice_kb*/ 32, /*c4_group_mi*/ 128, /*delta_enc_vec*/ 1,
    /*dscan*/ 1,          /*dscan_nt*/ 2,      /*fspec*/ 1,           /*fastdiv*/ 1,
    /*crc_lds*/ 0,        /*delta_enc_dv*/ 4,      /*br_planes*/ 1,       /*ck_fused_plain*/ 0,
};

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

static inline uint64_t mc_now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

// Spin on the verdict word for at most MC_VERDICT_SPIN_NS (a lone verify of
// 256 MiB is ~45 us, so the usual call never leaves the spin); a verify queued
// behind a lot of earlier work then keeps polling with a sleep between polls
// instead of holding a host core at 100 % for as long as the stream takes.
// (No hipStreamSynchronize: on the legacy default stream that would also wait
// for every other blocking stream's work, not just the verify.)
#define MC_VERDICT_SPIN_NS 100000ull
#define MC_VERDICT_SLEEP_NS 20000l

int mc_verdict_wait(const uint32_t *rec, uint32_t seq, mc_stream_t stream) {
  if (!rec || !seq) return MC_EINVAL;
  const uint64_t t0 = mc_now_ns();
  bool sleeping = false;
  for (unsigned i = 1;; ++i) {
    if (__atomic_load_n(&rec[2], __ATOMIC_ACQUIRE) == seq) return MC_OK;
    if (sleeping || (i & 1023u) == 0) {  // every ~10-20 us: has the stream ended or failed?
      const hipError_t e = hipStreamQuery((hipStream_t)stream);
      if (e == hipSuccess)
        return __atomic_load_n(&rec[2], __ATOMIC_ACQUIRE) == seq ? MC_OK : MC_EPROTO;
      if (e != hipErrorNotReady) return mc_hip_status(e);
      if (!sleeping) sleeping = mc_now_ns() - t0 > MC_VERDICT_SPIN_NS;
    }
    if (sleeping) {
      const timespec ts{0, MC_VERDICT_SLEEP_NS};
      nanosleep(&ts, nullptr);
    } else {
      __builtin_ia32_pause();
    }
  }
}

int mc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
