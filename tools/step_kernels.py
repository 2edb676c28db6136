"""Per-step kernel table from a rocprofv3 kernel_trace.csv: kernels launched between the
last two optimizer kernels (adam_ema_dev) of the run, i.e. exactly one train step."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
marks = [i for i, r in enumerate(rows) if 'adam_ema' in r['Kernel_Name']]
a, b = marks[-2], marks[-1]
step = rows[a + 1:b + 1]
agg = collections.defaultdict(lambda: [0, 0])
for r in step:
    n = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name'])
    n = re.sub(r'\(.*$', '', n) if not n.startswith('void at::') else n[:90]
    agg[n][0] += 1
    agg[n][1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
span = (int(step[-1]['End_Timestamp']) - int(step[0]['Start_Timestamp'])) / 1e6
busy = sum(v[1] for v in agg.values()) / 1e6
print(f'step span {span:.2f} ms, kernel busy {busy:.2f} ms, {len(step)} launches')
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f'{t / 1e6:8.3f} ms {c:5d} x {t / c / 1e3:8.1f} us  {n[:110]}')
