"""Per-phase clock cycles of the row-band forward kernel (diagnostics).

Runs conv_fwd_raw at one shape under a band variant with sr_conv3x3_set_stamps on and prints,
averaged over blocks: kernel-entry -> weights-loaded, loop total, and per-row cycles of the
row wait / barrier / MFMA / epilogue phases (wave 0's view).
usage: python tools/band_stamps.py B variant[,variant...] cin,cout,hw
"""
import json
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def main():
    B = int(sys.argv[1])
    variants = [int(v) for v in sys.argv[2].split(',')]
    cin, cout, hw = (int(v) for v in sys.argv[3].split(','))
    dev = 'cuda'
    lib = C._lib.load()
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(dev)
    spec = C.ConvSpec(cin, cout)
    x = torch.randn(B, hw, hw, C.pad8(cin), device=dev).to(torch.bfloat16)
    wf, wd, bg = C.prepared(conv.weight, conv.bias, spec, torch.bfloat16)
    y = torch.empty(B, hw, hw, C.pad8(cout), device=dev, dtype=torch.bfloat16)
    st = torch.zeros(256 * 16, device=dev, dtype=torch.int64)
    for v in variants:
        C._lib.check(lib.sr_conv3x3_set_variant(v))
        for _ in range(3):
            C.conv_fwd_raw(x, wf, bg, y, B, hw, hw, spec.cin_p, spec.cout_p, cout)
        st.zero_()
        C._lib.check(lib.sr_conv3x3_set_stamps(st.data_ptr()))
        C.conv_fwd_raw(x, wf, bg, y, B, hw, hw, spec.cin_p, spec.cout_p, cout)
        torch.cuda.synchronize()
        C._lib.check(lib.sr_conv3x3_set_stamps(None))
        s = st.view(256, 16).cpu()
        s = s[s[:, 3] > 0].double()
        rows = s[:, 3]
        out = dict(v=v, blocks=int(s.shape[0]), rows_per_block=float(rows.mean()),
                   load_cyc=float((s[:, 1] - s[:, 0]).mean()), zero_cyc=float((s[:, 8] - s[:, 0]).mean()),
                   wissue_cyc=float((s[:, 9] - s[:, 8]).mean()), wwait_cyc=float((s[:, 1] - s[:, 9]).mean()), loop_cyc=float((s[:, 2] - s[:, 1]).mean()),
                   loop_per_row=float(((s[:, 2] - s[:, 1]) / rows).mean()),
                   per_row=dict(wait=float((s[:, 4] / rows).mean()), barrier=float((s[:, 5] / rows).mean()),
                                mfma=float((s[:, 6] / rows).mean()), epilogue=float((s[:, 7] / rows).mean())))
        print(json.dumps(out), flush=True)
    C._lib.check(lib.sr_conv3x3_set_variant(0))


if __name__ == '__main__':
    main()
