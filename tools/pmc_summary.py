"""Fold one workload's rocprofv3 passes (tools/profile_round.sh) into profiles/.

Writes profiles/<tag>/<workload>_kernel_stats.csv (the --stats summary as rocprofv3 wrote
it), profiles/<tag>/<workload>_pmc.json (per-launch FETCH/WRITE of the dominant kernel) and
merges the per-launch HBM traffic into profiles/pmc_traffic.json, which bench.py reports as
``roofline.traffic``.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE counts half the bytes of 16-B/lane streaming reads (global_load and
buffer_load ... lds alike), so it is doubled; WRITE_SIZE is exact for 16-B/lane stores.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

tag, workload, kre, out, bench_kernel = sys.argv[1:6]  # bench_kernel: bench.py's ktrace name
# time / traffic regex: for a bench span that is a kernel + its slab reduce ('...+reduce'), both
# kernels' time and bytes per call of the kernel matching kre (default: kre itself)
tre = sys.argv[6] if len(sys.argv) > 6 else kre
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, 'profiles', tag)
os.makedirs(dst, exist_ok=True)

stats = glob.glob(os.path.join(out, 'kt', '**', '*kernel_stats.csv'), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, f'{workload}_kernel_stats.csv'))


def per_launch(pass_dir, counter):
    """Counter total over the kernels matching tre, per launch of the kernels matching kre."""
    tot, n, names = 0.0, 0, set()
    for f in glob.glob(os.path.join(out, pass_dir, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != counter:
                continue
            if re.search(tre, r['Kernel_Name']):
                tot += float(r['Counter_Value'])
                names.add(r['Kernel_Name'])
            if re.search(kre, r['Kernel_Name']):
                n += 1
    return (tot / n if n else None), n, sorted(names)


fetch_kib, nf, names = per_launch('fetch', 'FETCH_SIZE')
write_kib, nw, _ = per_launch('write', 'WRITE_SIZE')
avg_us = None
if stats:
    rows = list(csv.DictReader(open(stats[0])))
    calls = sum(int(r['Calls']) for r in rows if re.search(kre, r['Name']))
    if calls:
        avg_us = sum(float(r['TotalDurationNs']) for r in rows if re.search(tre, r['Name'])) / calls / 1e3
rec = {
    'kernel_regex': kre, 'time_regex': tre, 'bench_kernel': bench_kernel, 'kernels': names,
    'launches_counted': [nf, nw], 'stats_file': f'profiles/{tag}/{workload}_kernel_stats.csv',
    'fetch_size_kib_raw': fetch_kib, 'write_size_kib': write_kib,
    'fetch_bytes': None if fetch_kib is None else fetch_kib * 1024 * 2,
    'write_bytes': None if write_kib is None else write_kib * 1024,
    'rocprof_avg_us': avg_us,
    'correction': 'FETCH_SIZE KiB x1024 x2 (gfx950 half-count of 16-B/lane reads); WRITE_SIZE KiB x1024',
}
rec['hbm_bytes_per_launch'] = (None if rec['fetch_bytes'] is None or rec['write_bytes'] is None
                               else rec['fetch_bytes'] + rec['write_bytes'])
json.dump(rec, open(os.path.join(dst, f'{workload}_pmc.json'), 'w'), indent=1)
tp = os.path.join(root, 'profiles', 'pmc_traffic.json')
allrec = json.load(open(tp)) if os.path.exists(tp) else {}
allrec[workload] = dict(rec, source=f'profiles/{tag}/{workload}_pmc.json')
json.dump(allrec, open(tp, 'w'), indent=1, sort_keys=True)
print(workload, json.dumps(rec))
