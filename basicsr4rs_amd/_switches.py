"""Process-wide switches of the Python side, read from the environment here and nowhere else (the
Python twin of the library's knob table, csrc/sr_core.hip).  Module-level flags take their value at
import; ``switch`` itself reads the environment at each call (a spawned test worker sets
SR_ASYNC_WGRAD after importing the package, before it builds its model).  Each is an A/B or diagnostic
switch with the production default; DESIGN.md cites the measurements behind the defaults.

SR_HIP_LIB            path of libsr_hip.so (two-build A/B, tools/ab.sh)
SR_CONV_VARIANT       process-wide kernel-selection variant of the conv library (0: automatic)
SR_ASYNC_WGRAD        0 / 1 / reduce: overrides train.async_wgrad (side-stream weight gradients)
SR_SIDE_BATCH         blocks per side-stream fork (overrides train.async_wgrad_blocks)
SR_STB_SIDE_BATCH     0: SwinIR blocks fork their side-stream launches one by one
SR_PARAM_REDUCE_MAIN  1: LayerNorm / attention-table gradient reduces on the main stream
SR_ROWSCALE_UNFUSED   1: the proj-branch DropPath gradient by a separate row-scale pass
SR_SWIN_FUSED         0: a SwinIR block's attention half as three launches
SR_LN_UNFUSED         1 / qkv / fc1: the standalone LayerNorm kernel + linear instead of the LN-prologue linear
SR_CA_UNFUSED         1: the round-2 channel-attention launches
SR_CA_DOT             1: channel-attention dots from the next block's dgrad epilogue (measured slower, A/B)
SR_DCN_BWD_FUSED      0: the DCN backward through the dcols matrix
SR_CONV_KPAD          0: no K-padded weight images for the 184-channel 3x3 convs (the 64-channel halo kernel)
SR_STEP_TRACE         host time stamps of the segmented DDP graph step (a file path)
"""
import os

_DEFAULTS = {
    'SR_HIP_LIB': None,
    'SR_CONV_VARIANT': '0',
    'SR_ASYNC_WGRAD': None,
    'SR_SIDE_BATCH': None,
    'SR_STB_SIDE_BATCH': '1',
    'SR_PARAM_REDUCE_MAIN': '0',
    'SR_ROWSCALE_UNFUSED': '0',
    'SR_SWIN_FUSED': '1',
    'SR_LN_UNFUSED': None,
    'SR_CA_UNFUSED': '0',
    'SR_CA_DOT': '0',
    'SR_DCN_BWD_FUSED': '1',
    'SR_CONV_KPAD': '1',
    'SR_STEP_TRACE': None,
}


def switch(name):
    """The value of a switch (a string, or None when unset and without a default)."""
    return os.environ.get(name, _DEFAULTS[name])
