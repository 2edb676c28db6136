// Host-side helpers shared by the C-ABI entry points (error reporting).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/sr_hip.h"

int sr_fail(int code, const char* msg);
int sr_check(hipError_t e, const char* what);
