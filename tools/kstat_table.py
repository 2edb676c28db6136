"""Per-step table of a rocprofv3 kernel_stats.csv: ms / step, launches / step, average us, kernel.
usage: python3 tools/kstat_table.py <kernel_stats.csv> [steps (default: adam launches)] [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != '0' else \
    [int(r['Calls']) for r in rows if 'adam_ema' in r['Name']][0]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r['TotalDurationNs']) for r in rows) / steps / 1e6
print(f'steps {steps}, kernel time {tot:.2f} ms / step')
for r in rows[:top]:
    n = r['Name']
    n = n[n.find('::') + 2:] if '::' in n else n
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms {int(r['Calls']) / steps:7.1f}/step {float(r['AverageNs']) / 1e3:9.1f} us  {n[:110]}")
