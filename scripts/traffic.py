"""HBM traffic per dispatch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(run separately: scripts/gpu_pmc.sh), corrected as MI355X_MICROARCH.md
(HBM section) prescribes: FETCH_SIZE (KiB) counts wide 16-B/lane reads at
half their bytes on gfx950 -> x2; WRITE_SIZE (KiB) is exact for 16-B stores.

    python scripts/traffic.py gpurun_out/pmc [--envs 256 --t-max 5 --arch ff] > profiles/traffic_r02_c2.json
(the file records the source version it was measured on; bench.py uses a
traffic file only when that matches the tree it runs -- bench.source_version)
"""
import argparse
import re
import csv
import json
import os
from collections import defaultdict


def kernel_key(name: str) -> str:
    """'void arl::gemm_kernel<32, 64, ..., arl::EpiSlab, 2, 2>(...)' ->
    'gemm_kernel<32, 64, ..., EpiSlab, 2, 2>' (template instances stay apart)."""
    name = name.strip().replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    cut = [i for i in (name.find("<"), name.find("(")) if i >= 0]
    head = name[:min(cut)] if cut else name
    base = head.split("::")[-1]
    if cut and name[min(cut)] == "<":
        depth, end = 0, len(name)
        for i in range(min(cut), len(name)):
            depth += {"<": 1, ">": -1}.get(name[i], 0)
            if depth == 0:
                end = i + 1
                break
        base += re.sub(r"\b\w+::", "", name[min(cut):end])
    return base


def per_kernel(fn, counter):
    agg = defaultdict(list)
    for r in csv.DictReader(open(fn)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = kernel_key(name)
        agg[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--t-max", type=int, default=5)
    ap.add_argument("--arch", default="ff")
    ap.add_argument("--version", default=None, help="source version measured (default: this tree's, "
                                                        "bench.source_version)")
    a = ap.parse_args()
    if a.version is None:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import source_version
        a.version = source_version()
    fetch = per_kernel(os.path.join(a.pmc_dir, "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.pmc_dir, "write_counter_collection.csv"), "WRITE_SIZE")
    kernels, raw = {}, {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        raw[k] = {"FETCH_SIZE_KiB": round(f, 1), "WRITE_SIZE_KiB": round(w, 1)}
        kernels[k] = int(2 * f * 1024 + w * 1024)
    print(json.dumps({"envs": a.envs, "t_max": a.t_max, "arch": a.arch, "source_version": a.version,
                      "unit": "bytes per dispatch (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B)",
                      "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, --kernel-trace only",
                      "kernels": kernels, "raw": raw}, indent=1))


if __name__ == "__main__":
    main()
