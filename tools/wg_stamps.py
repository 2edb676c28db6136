"""Phase cycles of the row-streaming wgrad kernel (diagnostics; needs a -DSR_BAND_STAMPS build).
usage: python tools/wg_stamps.py B cin,cout,hw"""
import json
import sys

import torch

sys.path.insert(0, '.')
from basicsr4rs_amd.ops import conv as C  # noqa: E402


def main():
    B = int(sys.argv[1])
    cin, cout, hw = (int(v) for v in sys.argv[2].split(','))
    lib = C._lib.load()
    x = torch.randn(B, hw, hw, cin, device='cuda').to(torch.bfloat16)
    dy = torch.randn(B, hw, hw, cout, device='cuda').to(torch.bfloat16)
    st = torch.zeros(4096 * 16, device='cuda', dtype=torch.int64)
    for _ in range(3):
        C.conv_wgrad_raw(dy, x, B, hw, hw, cin, cin, cout, cout)
    C._lib.check(lib.sr_conv3x3_set_stamps(st.data_ptr()))
    C.conv_wgrad_raw(dy, x, B, hw, hw, cin, cin, cout, cout)
    torch.cuda.synchronize()
    C._lib.check(lib.sr_conv3x3_set_stamps(None))
    s = st.view(4096, 16).cpu()
    s = s[s[:, 3] > 0].double()
    nk = s[:, 3]
    print(json.dumps(dict(blocks=int(s.shape[0]), steps=float(nk.mean()), loop_cyc=float((s[:, 1] - s[:, 0]).mean()),
                          store_cyc=float((s[:, 2] - s[:, 1]).mean()),
                          per_step=dict(wait=float((s[:, 4] / nk).mean()), barrier1=float((s[:, 5] / nk).mean()),
                                        compute=float((s[:, 6] / nk).mean()), barrier2_issue=float((s[:, 7] / nk).mean())))))


if __name__ == '__main__':
    main()
