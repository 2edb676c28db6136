"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {int(r['Calls']):6d} calls {float(r['AverageNs']) / 1e3:10.1f} us"
          f"  {r['Name'][:120]}")
