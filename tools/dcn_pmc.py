"""Fold the DCN session's PMC passes (tools/r4_dcn.sh: one FETCH_SIZE and one WRITE_SIZE pass over
tools/bench_dcn.py --modes bf16) into profiles/<tag>/dcn_pmc.json: per DCN kernel, the per-launch
FETCH / WRITE bytes (median over its launches), next to the algorithmic bytes of the one definition
tools/bench_dcn.py uses (tensors once, as stored: x / dy bf16 NHWC, offset / mask and their
gradients, y and dx fp32).

Corrections (MI355X_MICROARCH.md, HBM section): WRITE_SIZE KiB x 1024 is exact for 16-B/lane
stores and float atomics.  FETCH_SIZE counts half the bytes of 16-B/lane streaming reads; the DCN
kernels mix those (x, dy, weights) with 4-B/lane reads (offsets, masks: most of the bytes), whose
count is uncalibrated, so both the raw KiB x 1024 and the x 2 figure are kept.

Usage: python tools/dcn_pmc.py gpurun_out/r4dcn r04
"""
import csv
import glob
import json
import os
import statistics
import sys

out, tag = sys.argv[1:3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MB = 1e6
N, C, H, W, DG, K = 16, 64, 128, 128, 8, 9
px = N * H * W
x_b, dy_b = 2 * px * C, 2 * px * C  # bf16 NHWC
om_b = 4 * px * DG * 3 * K  # offset (2 per tap) + mask (1 per tap), fp32
y_b, dx_b = 4 * px * C, 4 * px * C
ALG = {
    'dcn_fwd_win_kernel': (x_b + om_b + y_b, 'x bf16 + offset/mask fp32 in, y fp32 out (columns, when stored '
                                              'for the backward, are not algorithmic)'),
    'dcn_coord_dy8_kernel': (x_b + dy_b + 2 * om_b, 'x, dy bf16 + offset/mask fp32 in, their gradients out'),
    'dcn_gradx_dy8_kernel': (dy_b + om_b + dx_b, 'dy bf16 + offset/mask fp32 in, dx fp32 out'),
    'dcn_coord_win_kernel': (x_b + 2 * om_b, 'dcols path: x + offset/mask in, gradients out (dcols not counted)'),
    'dcn_grad_x_kernel': (om_b + dx_b, 'dcols path: offset/mask in, dx out (dcols not counted)'),
}


def short(name):
    for k in ALG:
        if k in name:
            return k
    return None


def collect(counter):
    """Per kernel, the counter of each launch in launch order."""
    vals = {}
    for f in glob.glob(os.path.join(out, f'pmc_{counter}', '**', '*counter_collection.csv'), recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Dispatch_Id']))
        for r in rows:
            if r['Counter_Name'] != counter:
                continue
            k = short(r['Kernel_Name'])
            if k:
                vals.setdefault(k, []).append(float(r['Counter_Value']) * 1024)
    return vals


fetch, write = collect('FETCH_SIZE'), collect('WRITE_SIZE')
# the forward runs both without (inference: y only) and with the columns stored for the backward
# (training: + 302 MB); the two passes launch in the same order, so split both by the WRITE size
k = 'dcn_fwd_win_kernel'
if k in write and k in fetch and len(write[k]) == len(fetch[k]):
    tr = [w > 200e6 for w in write[k]]
    for name, sel in (('dcn_fwd_win_kernel (training: + columns)', True), ('dcn_fwd_win_kernel (inference)', False)):
        fetch[name] = [f for f, t in zip(fetch[k], tr) if t == sel]
        write[name] = [w for w, t in zip(write[k], tr) if t == sel]
    del fetch[k], write[k]
    ALG['dcn_fwd_win_kernel (training: + columns)'] = (ALG[k][0], ALG[k][1] + '; 302 MB of columns written')
    ALG['dcn_fwd_win_kernel (inference)'] = ALG[k]
res = {'config': 'C5 op: x[16,64,128,128] offset[16,144,128,128] mask[16,72,128,128] W[64,64,3,3] dg 8, bf16',
       'correction': __doc__.split('Corrections')[1].split('Usage')[0].strip()}
for k, (alg, what) in ALG.items():
    if k not in fetch and k not in write:
        continue
    f = fetch.get(k, [])
    w = write.get(k, [])
    rec = {'algorithmic_MB': round(alg / MB, 1), 'algorithmic': what, 'launches': [len(f), len(w)]}
    if f:
        rec['fetch_MB_raw_median'] = round(statistics.median(f) / MB, 1)
        rec['fetch_MB_x2_median'] = round(2 * statistics.median(f) / MB, 1)
        rec['fetch_MB_raw_all'] = sorted(round(v / MB, 1) for v in f)
    if w:
        rec['write_MB_median'] = round(statistics.median(w) / MB, 1)
        rec['write_MB_all'] = sorted(round(v / MB, 1) for v in w)
    res[k] = rec
os.makedirs(os.path.join(root, 'profiles', tag), exist_ok=True)
json.dump(res, open(os.path.join(root, 'profiles', tag, 'dcn_pmc.json'), 'w'), indent=1)
print(json.dumps(res, indent=1))
