"""Phase cycles of the fused attention kernel (swin_attn_block_fwd_kernel, SR_SWIN_ATTN_DBG=32:
s_memtime stamps, the plain schedule otherwise unchanged) at the C4 bench shape (SwinIR-M, B 32,
64x64 tokens): per block, waves 0 and 4, averaged over blocks: LayerNorm prologue, step A, S1 wait,
step B, S2 wait, step C (summed over the 6 heads), total.  usage: python tools/swin_attn_stamps.py"""
import json
import sys

import torch

sys.path.insert(0, '.')
import bench  # noqa: E402
from basicsr4rs_amd import _lib  # noqa: E402


def main():
    from basicsr4rs_amd.archs import build_network
    from basicsr4rs_amd.ops import swin as S
    cfg = bench.WORKLOADS['swinir'][0]
    torch.manual_seed(0)
    net = build_network(dict(cfg)).cuda()
    blk = net._blocks()[1]
    at, g = blk.attn, blk._geom
    Cp = blk._fc1.cin_p
    x = torch.randn(32, 64, 64, Cp, device='cuda').to(torch.bfloat16)
    x[..., g.dim:] = 0
    qwf, _, qbg = S.prepared_linear(at.qkv.weight, at.qkv.bias, g.qkv, torch.bfloat16)
    pwf, _, pbg = S.prepared_linear(at.proj.weight, at.proj.bias, g.proj, torch.bfloat16)
    tab = at.relative_position_bias_table.detach().float().contiguous()
    nblk = 32 * 64 // 2
    st = torch.zeros(nblk * 16, device='cuda', dtype=torch.int64)
    lib = _lib.load()
    names = ['ln', 'A', 'S1wait', 'B', 'S2wait', 'C', 'total']
    for train in (True, False):
        with torch.no_grad():
            for _ in range(3):
                S.swin_attn_fused(x, blk.norm1.weight, blk.norm1.bias, g.dim, qwf, qbg, tab, pwf, pbg, None, g,
                                  float(at.scale), train)
            st.zero_()
            _lib.check(lib.sr_conv3x3_set_stamps(st.data_ptr()))
            try:
                with _lib.knob('SR_SWIN_ATTN_DBG', 32):
                    S.swin_attn_fused(x, blk.norm1.weight, blk.norm1.bias, g.dim, qwf, qbg, tab, pwf, pbg, None, g,
                                      float(at.scale), train)
                torch.cuda.synchronize()
            finally:
                _lib.check(lib.sr_conv3x3_set_stamps(None))
        v = st.view(nblk, 2, 8)[:, :, :7].double().cpu()
        for wv in (0, 1):
            m = v[:, wv].mean(0)
            print(json.dumps({'train': train, 'wave': 4 * wv,
                              **{n: round(m[i].item()) for i, n in enumerate(names)}}), flush=True)


if __name__ == '__main__':
    main()
