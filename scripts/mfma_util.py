"""Per-kernel MFMA utilisation from a rocprofv3 --pmc pass (gpu_mfma_pmc.sh).

util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM over the 8 XCDs; MI355X_MICROARCH.md
DVFS note), SIMDs = 256 CUs x 4.  SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy
SIMD cycles summed over the chip (32 per v_mfma_f32_16x16x4_f32 issue).
    python scripts/mfma_util.py <counter_collection.csv> [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict

SIMDS = 256 * 4
rows = defaultdict(lambda: defaultdict(list))
for fn in [a for a in sys.argv[1:] if a.endswith(".csv")]:
    for r in csv.DictReader(open(fn)):
        key = (r["Kernel_Name"], r.get("Dispatch_Id", ""))
        rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = defaultdict(list)
for (name, _), cs in rows.items():
    c = {k: sum(v) for k, v in cs.items()}
    if c.get("GRBM_GUI_ACTIVE", 0) <= 0:
        continue
    cyc = c["GRBM_GUI_ACTIVE"] / 8.0
    per[name].append({"util": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (SIMDS * cyc), "cycles": cyc,
                      "mfma_insts": c.get("SQ_INSTS_MFMA", 0.0), "valu_insts": c.get("SQ_INSTS_VALU", 0.0),
                      "lds_insts": c.get("SQ_INSTS_LDS", 0.0), "waves": c.get("SQ_WAVES", 0.0)})
out = {}
for name, lst in sorted(per.items(), key=lambda kv: -sum(d["cycles"] for d in kv[1])):
    n = len(lst)
    avg = {k: sum(d[k] for d in lst) / n for k in lst[0]}
    if avg["mfma_insts"] == 0:
        continue
    short = name.replace("(anonymous namespace)::", "").split("(")[0][:90]
    out[short] = {"dispatches": n, "mfma_busy_frac": round(avg["util"], 4), "cycles": round(avg["cycles"]),
                  "mfma_insts": round(avg["mfma_insts"]), "valu_insts": round(avg["valu_insts"]),
                  "lds_insts": round(avg["lds_insts"]), "waves": round(avg["waves"])}
    print(f"{avg['util'] * 100:6.1f}%  cyc={avg['cycles']:9.0f}  mfma={avg['mfma_insts']:10.0f}  n={n:3d}  {short}")
if "--json" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
