// Host-side helpers shared by the C-ABI entry points (error reporting, tuning knobs).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/sr_hip.h"

int sr_fail(int code, const char* msg);
int sr_check(hipError_t e, const char* what);

// Tuning knobs (sr_core.hip): environment variable of the same name read once per process,
// overridable by sr_set_knob; -1 = unset.
enum SrKnob {
  K_LWK,            // SR_LWK=0: linears on the lin kernel instead of linear_wk_kernel (A/B)
  K_LWK_MINK,       // SR_LWK_MINK: linear_wk_kernel only for K above this
  K_RING_WIDE,      // SR_RING_WIDE: 0 off / > 0 block target of the row-streaming wgrad over 64-co tiles
  K_RING_PS,        // SR_RING_PS=0: pixel-shuffled dy off the ring wgrad (A/B)
  K_LWG,            // SR_LWG=0: 1x1 wgrads on the pp kernel instead of linear_wgrad_kernel (A/B)
  K_LWG_T,          // SR_LWG_T: block target of the linear_wgrad split plan
  K_RING_SPLITS,    // SR_RING_SPLITS: block target of the narrow ring wgrad split plan
  K_DCN_CPP,        // SR_DCN_CPP: channels per pass of the DCN scatter
  K_DCN_DBG,        // SR_DCN_DBG: DCN forward timing ablations (wrong results)
  K_DCN_R,          // SR_DCN_R: x-window margin of the fused DCN forward
  K_DCN_FUSED,      // SR_DCN_FUSED=0: unfused DCN forward (A/B)
  K_DCN_COORD_WIN,  // SR_DCN_COORD_WIN=0: global-memory coordinate gradients (A/B)
  K_DCN_GX_FX,      // SR_DCN_GX_FX: 32 / 64-bit fixed-point scatter image
  K_SWIN_ATTN_DBG,  // SR_SWIN_ATTN_DBG: fused attention timing ablations (wrong results)
  K_WG_ROW3,        // SR_WG_ROW3: 0 = the kernel-row wgrad off (pp kernel), > 0 = its bias-role group size
  K_COUNT
};
int sr_knob(SrKnob k);
// diagnostics buffer of per-block clock stamps (sr_conv3x3_set_stamps; null = off)
extern unsigned long long* g_sr_stamps;
