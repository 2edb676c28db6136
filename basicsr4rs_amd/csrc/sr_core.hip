// Library identity, thread-local error reporting and the tuning knobs for the C ABI (include/sr_hip.h).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <mutex>
#include "sr_internal.h"

static thread_local char g_err[512] = "";
unsigned long long* g_sr_stamps = nullptr;

int sr_fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int sr_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return SR_OK;
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
  return SR_ELAUNCH;
}

// Tuning knobs (A/B switches and plan targets).  Each is read from its environment variable ONCE
// per process (the library's only getenv site) and can be overridden at run time by sr_set_knob;
// kernels read the cached value (no per-call environment lookups).  -1 = unset (the built-in default).
static const char* const kKnobNames[K_COUNT] = {
    "SR_LWK", "SR_LWK_MINK", "SR_RING_WIDE", "SR_RING_PS", "SR_LWG", "SR_LWG_T", "SR_RING_SPLITS",
    "SR_DCN_CPP", "SR_DCN_DBG", "SR_DCN_R", "SR_DCN_FUSED", "SR_DCN_COORD_WIN",
    "SR_DCN_GX_FX", "SR_SWIN_ATTN_DBG", "SR_WG_ROW3"};
static std::atomic<int> g_knob[K_COUNT];
static std::once_flag g_knob_once;

static void knob_init() {
  for (int k = 0; k < K_COUNT; ++k) {
    const char* e = getenv(kKnobNames[k]);
    g_knob[k].store(e && *e ? atoi(e) : -1, std::memory_order_relaxed);
  }
}

int sr_knob(SrKnob k) {
  std::call_once(g_knob_once, knob_init);
  return g_knob[k].load(std::memory_order_relaxed);
}

static int knob_index(const char* name) {
  if (!name) return -1;
  for (int k = 0; k < K_COUNT; ++k)
    if (strcmp(kKnobNames[k], name) == 0) return k;
  return -1;
}

extern "C" int sr_set_knob(const char* name, int value, int* previous) {
  const int k = knob_index(name);
  if (k < 0) return sr_fail(SR_EINVAL, "set_knob: unknown knob name");
  std::call_once(g_knob_once, knob_init);
  const int old = g_knob[k].exchange(value < 0 ? -1 : value, std::memory_order_relaxed);
  if (previous) *previous = old;
  return SR_OK;
}

extern "C" int sr_get_knob(const char* name) {
  const int k = knob_index(name);
  return k < 0 ? -2 : sr_knob((SrKnob)k);
}

extern "C" const char* sr_version(void) { return "basicsr4rs_amd libsr_hip 0.2 (gfx950)"; }
extern "C" const char* sr_last_error(void) { return g_err; }
