"""Average PMC counters of one kernel (name substring) from a rocprofv3 --pmc
output directory; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8)."""
import collections
import csv
import glob
import sys

d, name = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if name in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = list(agg.values())
avg = {k: sum(x[k] for x in rows) / len(rows) for k in rows[0]}
print(name, {k: round(v) for k, v in avg.items()})
if "GRBM_GUI_ACTIVE" in avg and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
    print("mfma busy %.3f" % (avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * avg["GRBM_GUI_ACTIVE"] / 8)))
