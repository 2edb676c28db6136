// Library identity and thread-local error reporting for the C ABI (include/sr_hip.h).
#include <stdio.h>
#include <string.h>
#include "sr_internal.h"

static thread_local char g_err[512] = "";

int sr_fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int sr_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return SR_OK;
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
  return SR_ELAUNCH;
}

extern "C" const char* sr_version(void) { return "basicsr4rs_amd libsr_hip 0.1 (gfx950)"; }
extern "C" const char* sr_last_error(void) { return g_err; }
