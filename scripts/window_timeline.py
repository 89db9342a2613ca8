"""Per-window timeline from a rocprofv3 kernel trace of bench.py: kernel
durations, the idle gaps between consecutive kernels and the window period,
averaged over the timed graph replays (windows start at the first kernel after
rmsprop_kernel).
    python scripts/window_timeline.py gpurun_out/<tag>/prof/run_kernel_trace.csv"""
import csv
import re
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("arl::", "")
        name = name.replace("(anonymous namespace)::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
# windows = runs of kernels ending with rmsprop_kernel; keep runs whose kernel sequence is the most common one
wins, cur = [], []
for r in rows:
    cur.append(r)
    if r[2].startswith("rmsprop_kernel"):
        wins.append(cur)
        cur = []
seqs = defaultdict(list)
for w in wins:
    # drop the leading kernels that belong to the previous window's tail / setup
    seqs[tuple(k for _, _, k in w)].append(w)
seq, ws = max(((k, v) for k, v in seqs.items() if len(k) > 8), key=lambda kv: len(kv[1]))
print(f"{len(ws)} windows of {len(seq)} kernels")
n = len(seq)
dur = [0.0] * n
gap = [0.0] * n
per = []
for w in ws:
    for i, (s, e, k) in enumerate(w):
        dur[i] += (e - s) / 1e3
        if i:
            gap[i] += (s - w[i - 1][1]) / 1e3
    per.append((w[-1][1] - w[0][0]) / 1e3)
m = len(ws)
for i, k in enumerate(seq):
    print(f"{i:2d} {k[:60]:60s} {dur[i] / m:7.2f} us  gap before {gap[i] / m:6.2f}")
print(f"sum kernels {sum(dur) / m:.1f} us, sum gaps {sum(gap) / m:.1f} us, first->last {sum(per) / m:.1f} us")
