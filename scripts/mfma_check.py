"""Checks bench.py's matrix-pipe model (mfma_cycles) against the counters.

For one workload's rocprofv3 --pmc pass (gpu_mfma_pmc.sh: SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_MFMA, GRBM_GUI_ACTIVE with --kernel-trace) this prints, per MFMA
kernel, the model's issued matrix cycles per launch next to the counter's,
and the utilisations of the same dispatches:
  frac_issued       = model cycles / (SIMDs x 2.4 GHz x the traced duration)   (bench.py's)
  busy_frac_traced  = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x 2.4 GHz x the traced duration)
  busy_frac_grbm    = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / 8): GRBM's window also
                      holds the profiler's per-dispatch counter start / stop (several us on short kernels)
    python scripts/mfma_check.py <dir with *counter_collection.csv, *kernel_trace.csv> \
        --workload c4 [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

STAGE_OF = [("conv_fwd_kernel", "conv_fwd"), ("fc_fwd_kernel", "fc_fwd"), ("conv_bwd_kernel", "conv_bwd"),
            ("conv_bwd_ws_kernel", "conv_bwd"),
            ("lstm_gates_kernel", "lstm_gates"), ("lstm_bptt_kernel", "lstm_bptt")]


def stage_of(name):
    if "reduce_conv_bwd" in name:
        return None
    if "fc_bwd_kernel" in name:
        return "lstm_wgrad" if "ShapeLSTM" in name else "fc_bwd"
    for k, v in STAGE_OF:
        if k in name:
            return v
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    arch, N, _ = bench.WORKLOADS[a.workload]
    T = 5
    ctr = defaultdict(lambda: defaultdict(float))
    names = {}
    for fn in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            d = r["Dispatch_Id"]
            ctr[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    dur = {}
    for fn in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(list)
    for d, c in ctr.items():
        st = stage_of(names[d])
        if st is None or c.get("GRBM_GUI_ACTIVE", 0) <= 0 or d not in dur:
            continue
        per[st].append((c, dur[d]))
    out = {}
    for st, lst in sorted(per.items()):
        model = bench.mfma_cycles(st, N, T, "lstm" if arch.endswith("lstm") else "ff")
        n = len(lst)
        busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c, _ in lst) / n
        insts = sum(c["SQ_INSTS_MFMA"] for c, _ in lst) / n
        kcyc = sum(c["GRBM_GUI_ACTIVE"] / 8.0 for c, _ in lst) / n
        t = sum(x for _, x in lst) / n
        fi = model / (bench.SIMDS * bench.CLK_HZ * t)
        bf = busy / (bench.SIMDS * kcyc)
        bt = busy / (bench.SIMDS * bench.CLK_HZ * t)   # the counter's cycles on the traced time base
        out[st] = {"dispatches": n, "model_cycles": model, "busy_cycles": busy, "model_over_busy": model / busy,
                   "mfma_insts": insts, "us": t * 1e6, "frac_issued": fi, "busy_frac_traced": bt,
                   "points_apart_traced": 100 * (fi - bt), "busy_frac_grbm": bf, "grbm_us": kcyc / bench.CLK_HZ * 1e6}
        print(f"{st:11s} n={n:3d} model={model:12.0f} busy={busy:12.0f} ratio={model / busy:6.3f} "
              f"insts={insts:10.0f} {t * 1e6:7.1f} us  frac_issued={fi:.3f} busy_frac_traced={bt:.3f} "
              f"({100 * (fi - bt):+.1f} pts)  busy_frac_grbm={bf:.3f} (GRBM window {kcyc / bench.CLK_HZ * 1e6:.1f} us)")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
