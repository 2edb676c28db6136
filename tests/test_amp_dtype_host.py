"""AMP dtype mapping: the reference's fp16 autocast + GradScaler
(basicsr/models/srrs_model.py:28-31, 79-82) runs as bf16 on the HIP kernels; an fp16 autocast
request warns once instead of silently switching.  Host test: autocast state is stubbed (CUDA
autocast is disabled without a GPU)."""
import warnings

import torch

from basicsr4rs_amd.ops import conv as C


def test_fp16_autocast_request_warns_once(monkeypatch):
    monkeypatch.setattr(C.torch, 'is_autocast_enabled', lambda dev='cuda': True)
    monkeypatch.setattr(C.torch, 'get_autocast_dtype', lambda dev='cuda': torch.float16)
    monkeypatch.setattr(C, '_FP16_WARNED', [False])
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        assert C.feature_dtype() == torch.bfloat16
        assert C.feature_dtype() == torch.bfloat16
    msgs = [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]
    assert len(msgs) == 1 and 'float16' in msgs[0] and 'bfloat16' in msgs[0]


def test_bf16_autocast_is_silent(monkeypatch):
    monkeypatch.setattr(C.torch, 'is_autocast_enabled', lambda dev='cuda': True)
    monkeypatch.setattr(C.torch, 'get_autocast_dtype', lambda dev='cuda': torch.bfloat16)
    monkeypatch.setattr(C, '_FP16_WARNED', [False])
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        assert C.feature_dtype() == torch.bfloat16
    assert not [x for x in w if issubclass(x.category, RuntimeWarning)]


def test_no_autocast_is_fp32(monkeypatch):
    monkeypatch.setattr(C.torch, 'is_autocast_enabled', lambda dev='cuda': False)
    assert C.feature_dtype() == torch.float32
