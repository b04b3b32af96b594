"""Top kernels of a rocprofv3 --stats csv by total time.  python tools/trace_top.py STATS.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}%  calls {int(r['Calls']):6d}  avg {float(r['AverageNs']) / 1e3:8.2f} us"
          f"  {r['Name'][:120]}")
print(f"total {tot / 1e6:.3f} ms")
