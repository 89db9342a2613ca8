"""Kernel statistics from a rocprofv3 --kernel-trace database (rocpd SQLite,
the default output format): per kernel the calls, average / min / max / total
duration, like rocprofv3's kernel_stats.csv, and, with --timeline <first
kernel substring>, the durations of one window's kernels in dispatch order
averaged over every occurrence of the window's kernel sequence.

    python scripts/kstats_db.py gpurun_out/r4b/prof/c4_results.db [--csv out.csv]
        [--timeline conv_fwd_kernel --window 28]
"""
import argparse
import csv
import re
import sqlite3
from collections import OrderedDict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    return name.replace("void ", "").replace("arl::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--timeline", help="substring of the kernel that opens a window")
    ap.add_argument("--window", type=int, default=0, help="kernels per window (0: up to the next opener)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    stats = OrderedDict()
    for name, t0, t1 in rows:
        k = short(name)
        st = stats.setdefault(k, [0, 0, 1 << 62, 0])
        dur = t1 - t0
        st[0] += 1
        st[1] += dur
        st[2] = min(st[2], dur)
        st[3] = max(st[3], dur)
    order = sorted(stats.items(), key=lambda kv: -kv[1][1])
    total = sum(v[1] for v in stats.values())
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>9s} {'min_us':>8s} {'max_us':>8s} {'pct':>6s}")
    for k, (n, tot, mn, mx) in order:
        print(f"{k[:70]:70s} {n:6d} {tot / n / 1e3:9.2f} {mn / 1e3:8.2f} {mx / 1e3:8.2f} {100 * tot / total:6.2f}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for k, (n, tot, mn, mx) in order:
                w.writerow([k, n, tot, tot / n, 100 * tot / total, mn, mx])
    if a.timeline:
        starts = [i for i, (name, _, _) in enumerate(rows) if a.timeline in name]
        wins = []
        for i0, i1 in zip(starts, starts[1:] + [len(rows)]):
            seg = rows[i0:i0 + a.window] if a.window else rows[i0:i1]
            wins.append(seg)
        # keep the windows whose kernel sequence is the most common one (the timed windows)
        sig = {}
        for wseg in wins:
            sig.setdefault(tuple(short(r[0]) for r in wseg), []).append(wseg)
        names, segs = max(sig.items(), key=lambda kv: len(kv[1]))
        print(f"\n{len(segs)} windows of {len(names)} kernels")
        tot_k = tot_g = 0.0
        for j, k in enumerate(names):
            d = sum(s[j][2] - s[j][1] for s in segs) / len(segs) / 1e3
            g = (sum(s[j][1] - s[j - 1][2] for s in segs) / len(segs) / 1e3) if j > 0 else 0.0
            tot_k += d
            tot_g += g
            print(f"{j:2d} {k[:60]:60s} {d:8.2f} us  gap before {g:6.2f}")
        print(f"sum kernels {tot_k:.1f} us, sum gaps {tot_g:.1f} us, first->last {tot_k + tot_g:.1f} us")


if __name__ == "__main__":
    main()
