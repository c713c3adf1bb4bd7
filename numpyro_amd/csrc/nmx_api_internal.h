// Error plumbing shared by the C-ABI entry points (status codes of include/numpyro_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/numpyro_amd.h"

int nmx_fail(int code, const char* fmt, ...);
int nmx_check_launch(const char* what);
// Raise `fn`'s dynamic-LDS limit to `bytes` on the device of `stream` (once per kernel and
// device; no-op at <= 64 KiB).  Returns NMX_OK or a status with nmx_last_error set.
int nmx_lds_limit(const void* fn, size_t bytes, hipStream_t stream, const char* what);
