"""Top kernels of a rocprofv3 --stats kernel_stats.csv: python scripts/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6} avg={float(r['AverageNs']) / 1000:8.2f}us "
          f"pct={float(r['Percentage']):6.2f}")
