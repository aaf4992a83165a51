// LAB ONLY: the vendor library's single-pass (decoupled look-back) scan,
// rocprim::inclusive_scan, over the same buffers as the integer Delta decode
// -- a yardstick for mc_delta_decode's two-launch scan
// (tools/probe_rocprim_scan.py), never part of libmcodec.so.
#include <cstring>

#include <rocprim/device/device_scan.hpp>

#include <cstdint>

namespace {

template <class T>
int scan(const void *src, void *dst, size_t n, void *ws, size_t *ws_bytes, hipStream_t st) {
  return (int)rocprim::inclusive_scan(ws, *ws_bytes, static_cast<const T *>(src), static_cast<T *>(dst), n,
                                      rocprim::plus<T>(), st, false);
}

int dispatch(int es, const void *src, void *dst, size_t n, void *ws, size_t *ws_bytes, hipStream_t st) {
  switch (es) {
    case 1:
      return scan<uint8_t>(src, dst, n, ws, ws_bytes, st);
    case 2:
      return scan<uint16_t>(src, dst, n, ws, ws_bytes, st);
    case 4:
      return scan<uint32_t>(src, dst, n, ws, ws_bytes, st);
    case 8:
      return scan<uint64_t>(src, dst, n, ws, ws_bytes, st);
    default:
      return -22;
  }
}

}  // namespace

// workspace bytes rocprim asks for (es = element bytes, unsigned wrap-around sums)
extern "C" size_t mc_lab_rocprim_scan_workspace(size_t n, int es) {
  size_t b = 0;
  if (dispatch(es, nullptr, nullptr, n, nullptr, &b, nullptr) != 0) return 0;
  return b;
}

extern "C" int mc_lab_rocprim_scan(const void *src, void *dst, size_t n, int es, void *ws, size_t ws_bytes,
                                   void *stream) {
  size_t b = ws_bytes;
  return dispatch(es, src, dst, n, ws, &b, (hipStream_t)stream);
}
