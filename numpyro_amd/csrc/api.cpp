// C-ABI housekeeping: version, error strings.  Kernel entry points live next to
// their kernels (nuts.hip, potential_*.hip, selftest.hip).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
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

extern "C" int nmx_version(void) { return NMX_VERSION; }

extern "C" const char* nmx_last_error(void) { return g_last_error; }

extern "C" size_t nmx_struct_size(int which) {
  switch (which) {
    case 0: return sizeof(nmx_nuts_config);
    case 1: return sizeof(nmx_eval_batch);
    default: return 0;
  }
}
