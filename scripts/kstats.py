"""Top kernels of a rocprofv3 --stats kernel_stats.csv: python scripts/kstats.py CSV [PASSES] [TOP]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
passes = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} us "
          f"{float(r['TotalDurationNs']) / passes / 1e6:8.3f} ms/pass")
print(f"total {tot / passes / 1e6:.3f} ms/pass")
