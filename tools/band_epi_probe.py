"""Time and phase-stamp the band kernel's epilogue forms at one shape (diagnostics).

For each epilogue ('plain', 'res', 'relu', 'colsum', 'res_dot'): the average launch time over 200
back-to-back launches (HIP events), and -- with a -DSR_BAND_STAMPS build (SR_HIP_LIB) -- wave 0's
per-row cycles of the row wait / barrier / MFMA / epilogue phases averaged over blocks.
usage: python tools/band_epi_probe.py B cin,cout,hw [epi,...]
"""
import json
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def main():
    B = int(sys.argv[1])
    cin, cout, hw = (int(v) for v in sys.argv[2].split(','))
    epis = sys.argv[3].split(',') if len(sys.argv) > 3 else ['plain', 'res', 'relu', 'colsum', 'res_dot']
    dev = 'cuda'
    lib = C._lib.load()
    dt = torch.bfloat16
    conv = torch.nn.Conv2d(cin, cout, 3, 1, 1).to(dev)
    spec = C.ConvSpec(cin, cout)
    x = torch.randn(B, hw, hw, cin, device=dev).to(dt)
    res = torch.randn(B, hw, hw, cout, device=dev).to(dt)
    dot = torch.randn(B, hw, hw, cout, device=dev).to(dt)
    wf, _, bg = C.prepared(conv.weight, conv.bias, spec, dt)
    y = torch.empty(B, hw, hw, cout, device=dev, dtype=dt)
    st = torch.zeros(256 * 16, device=dev, dtype=torch.int64)
    has_stamps = True
    for epi in epis:
        kw = {'plain': {}, 'res': dict(res=res, beta=1.0), 'relu': dict(act=1),
              'colsum': dict(colsum=True), 'res_dot': dict(res=res, beta=1.0, colsum=True, dot=dot)}[epi]

        def run():
            C.conv_fwd_raw(x, wf, bg if epi != 'res_dot' else None, y, B, hw, hw, cin, cout, cout, **kw)

        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            run()
        e1.record()
        torch.cuda.synchronize()
        out = dict(epi=epi, us=round(e0.elapsed_time(e1) * 1e3 / 200, 2))
        if has_stamps:
            st.zero_()
            try:
                C._lib.check(lib.sr_conv3x3_set_stamps(st.data_ptr()))
            except Exception:
                has_stamps = False
            if has_stamps:
                run()
                torch.cuda.synchronize()
                C._lib.check(lib.sr_conv3x3_set_stamps(None))
                s = st.view(256, 16).cpu()
                s = s[s[:, 3] > 0].double()
                if s.shape[0]:
                    rows = s[:, 3]
                    out.update(rows_per_block=float(rows.mean()), load_cyc=round(float((s[:, 1] - s[:, 0]).mean())),
                               loop_per_row=round(float(((s[:, 2] - s[:, 1]) / rows).mean())),
                               wait=round(float((s[:, 4] / rows).mean())), barrier=round(float((s[:, 5] / rows).mean())),
                               mfma=round(float((s[:, 6] / rows).mean())), epilogue=round(float((s[:, 7] / rows).mean())))
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
