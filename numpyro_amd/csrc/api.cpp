// C-ABI housekeeping: version, error strings.  Kernel entry points live next to
// their kernels (nuts.hip, potential_*.hip, selftest.hip).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <utility>

#include "nmx_api_internal.h"

static thread_local char g_last_error[512] = "";

int nmx_fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}

int nmx_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return nmx_fail(NMX_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return NMX_OK;
}

// hipFuncSetAttribute holds per device: a kernel launched on several GPUs of one process needs
// its dynamic-LDS limit raised on each.  Remembered per (kernel, device) so the host call is
// made once; the device is the launch stream's (the calling thread's current device may be
// another one).  Called on every launch of the hot kernels: a per-thread cache of the last
// (kernel, stream) answered is checked first, so the launch path takes no lock and makes no
// HIP call once a (kernel, stream) pair has been served (host threads of an in-process
// multi-device run never meet here after their first launches).
int nmx_lds_limit(const void* fn, size_t bytes, hipStream_t stream, const char* what) {
  if (bytes <= 64 * 1024) return NMX_OK;
  struct Hit {
    const void* fn;
    hipStream_t stream;
    size_t bytes;
  };
  static thread_local Hit hits[8] = {};
  static thread_local unsigned next_hit = 0;
  // (the null stream is the calling thread's current device, which may change: not cached)
  if (stream)
    for (const Hit& h : hits)
      if (h.fn == fn && h.stream == stream && h.bytes >= bytes) return NMX_OK;
  int dev = 0;
  hipError_t e = stream ? hipStreamGetDevice(stream, &dev) : hipGetDevice(&dev);
  if (e != hipSuccess) return nmx_fail(NMX_ERR_HIP, "%s: device of the stream: %s", what, hipGetErrorString(e));
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> done;
  std::lock_guard<std::mutex> lock(mu);
  auto it = done.find({fn, dev});
  if (it != done.end() && it->second >= bytes) {
    if (stream) hits[next_hit++ % 8] = Hit{fn, stream, it->second};
    return NMX_OK;
  }
  int cur = dev;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (cur != dev) (void)hipSetDevice(cur);
  if (e != hipSuccess) return nmx_fail(NMX_ERR_HIP, "%s: hipFuncSetAttribute: %s", what, hipGetErrorString(e));
  done[{fn, dev}] = bytes;
  if (stream) hits[next_hit++ % 8] = Hit{fn, stream, bytes};
  return NMX_OK;
}

extern "C" int nmx_version(void) { return NMX_VERSION; }

extern "C" const char* nmx_last_error(void) { return g_last_error; }

extern "C" size_t nmx_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(nmx_nuts_config);
    case 1: return sizeof(nmx_eval_batch);
    default: return 0;
  }
}
