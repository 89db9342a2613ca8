"""Per-kernel LDS and wait ratios from the gpu_stall_pmc.sh LDS pass:
  bank conflict  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS-array cycle)
  LDS wait       = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (wave cycles waiting on an LDS instruction)
  any wait       = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  LDS / VALU / MISC active = SQ_ACTIVE_INST_* / SQ_WAVE_CYCLES
Ratios of counters summed over the chip, averaged over a kernel's dispatches.
    python scripts/lds_util.py <counter_collection.csv> [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict

rows = defaultdict(lambda: defaultdict(float))
for fn in [a for a in sys.argv[1:] if a.endswith(".csv")]:
    for r in csv.DictReader(open(fn)):
        rows[(r["Kernel_Name"], r.get("Dispatch_Id", ""))][r["Counter_Name"]] += float(r["Counter_Value"])
per = defaultdict(list)
for (name, _), c in rows.items():
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0:
        continue
    per[name].append({
        "bank_conflict": c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c.get("SQ_LDS_IDX_ACTIVE", 0.0), 1.0),
        "lds_wait": c.get("SQ_WAIT_INST_LDS", 0.0) / wc,
        "any_wait": c.get("SQ_WAIT_ANY", 0.0) / wc,
        "lds_active": c.get("SQ_ACTIVE_INST_LDS", 0.0) / wc,
        "valu_active": c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
        "misc_active": c.get("SQ_ACTIVE_INST_MISC", 0.0) / wc,
        "gpu_cycles": c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0,
    })
out = {}
for name, lst in sorted(per.items(), key=lambda kv: -sum(d["gpu_cycles"] for d in kv[1])):
    n = len(lst)
    avg = {k: sum(d[k] for d in lst) / n for k in lst[0]}
    short = name.replace("(anonymous namespace)::", "").split("(")[0][:90]
    out[short] = {"dispatches": n, **{k: round(v, 4) for k, v in avg.items()}}
    print(f"conflict {avg['bank_conflict']:6.3f}  lds_wait {avg['lds_wait']:5.3f}  any_wait {avg['any_wait']:5.3f}  "
          f"lds {avg['lds_active']:5.3f}  valu {avg['valu_active']:5.3f}  cyc {avg['gpu_cycles']:9.0f}  n={n:3d}  {short}")
if "--json" in sys.argv:
    with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
        json.dump(out, f, indent=1)
