"""Registry semantics of basicsr/utils/registry.py:4-88 and the build_* surfaces."""
import pytest

from basicsr4rs_amd.utils.registry import ARCH_REGISTRY, LOSS_REGISTRY, METRIC_REGISTRY, MODEL_REGISTRY, Registry


def test_register_get_suffix_duplicate():
    r = Registry('t')

    @r.register()
    class A:
        pass

    r.register(A, suffix='x')
    assert r.get('A') is A
    assert 'A' in r and 'A_x' in r
    with pytest.raises(AssertionError):
        r.register(A)
    with pytest.raises(KeyError):
        r.get('missing')

    class C:
        pass

    r.register(C, suffix='basicsr')
    assert r.get('C') is C  # falls back to C_basicsr


def test_surfaces_registered():
    import basicsr4rs_amd.archs  # noqa: F401
    import basicsr4rs_amd.models  # noqa: F401
    assert 'EDSR' in ARCH_REGISTRY
    assert 'SRModel' in MODEL_REGISTRY
    assert 'L1Loss' in LOSS_REGISTRY
    assert 'calculate_psnr' in METRIC_REGISTRY


def test_edsr_state_dict_keys_match_reference_layout():
    """Keys/shapes of the reference EDSR (basicsr/archs/edsr_arch.py:40-48, arch_util.py:123-142)."""
    from basicsr4rs_amd.archs import build_network
    net = build_network(dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=2, upscale=4))
    sd = net.state_dict()
    expect = ['conv_first.weight', 'conv_first.bias']
    for i in range(2):
        expect += [f'body.{i}.conv1.weight', f'body.{i}.conv1.bias', f'body.{i}.conv2.weight', f'body.{i}.conv2.bias']
    expect += ['conv_after_body.weight', 'conv_after_body.bias', 'upsample.0.weight', 'upsample.0.bias',
               'upsample.2.weight', 'upsample.2.bias', 'conv_last.weight', 'conv_last.bias']
    assert list(sd.keys()) == expect
    assert sd['upsample.0.weight'].shape == (256, 64, 3, 3)
    net3 = build_network(dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=1, upscale=3))
    assert net3.state_dict()['upsample.0.weight'].shape == (576, 64, 3, 3)
    with pytest.raises(ValueError):
        build_network(dict(type='EDSR', num_in_ch=3, num_out_ch=3, num_feat=64, num_block=1, upscale=5))
