"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
for fn in sys.argv[1:]:
    for r in csv.DictReader(open(fn)):
        name = r["Kernel_Name"][:60]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v)/len(v):16.1f}   (n={len(v)})")
