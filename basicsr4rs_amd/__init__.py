"""basicsr4rs_amd — MI355X-native (gfx950) engine for the BasicSR4RS super-resolution hot path.

Drop-in for the reference's ``basicsr`` registries (ARCH_REGISTRY / MODEL_REGISTRY /
LOSS_REGISTRY): the SR nets (EDSR, RCAN, RRDBNet, SwinIR, MSRResNet) run their
forward/backward on hand-written HIP kernels (libsr_hip.so, include/sr_hip.h).
"""
__version__ = '0.1.0'
