"""Print the top kernels of a rocprofv3 --stats csv: share, calls, average duration.
    python tools/kstats.py gpurun_out/prw/run_kernel_stats.csv [N] [filter]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
flt = sys.argv[3] if len(sys.argv) > 3 else ''
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    if flt not in r['Name']:
        continue
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:120]}")
    n -= 1
    if n == 0:
        break
