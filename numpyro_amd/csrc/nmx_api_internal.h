// Error plumbing shared by the C-ABI entry points (status codes of include/numpyro_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/numpyro_amd.h"

int nmx_fail(int code, const char* fmt, ...);
int nmx_check_launch(const char* what);
