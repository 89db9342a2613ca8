"""Summarise a rocprofv3 kernel_stats.csv (per-kernel share of GPU time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{float(r['TotalDurationNs'])/tot*100:5.1f}% calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.2f}us  {r['Name'][:100]}")
print('total ms', round(tot / 1e6, 3))
