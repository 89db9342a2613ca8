"""Per-phase timeline of conv_bwd_kernel from an ARL_CB_STAMP build
(make -C async-rl_amd/csrc variant NAME=stamp DEFS="-DARL_CB_STAMP=1"):
s_memtime at every barrier, written into the slab (results wrong by design).
    ASYNCRL_HIP_LIB=.../build_var_stamp/libasyncrl_hip.so python scripts/cb_stamps.py
"""
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
import bench  # noqa: E402
from asyncrl_amd import A3C, A3CFF, RMSpropAsync  # noqa: E402

SLAB = 12336
SLAB_W1 = 8224
PH = ["commit", "step1+mask", "step2", "step3"]


def main():
    dev = torch.device("cuda", 0)
    N, T = int(os.environ.get("ENVS", "256")), 5
    model = A3CFF(4, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev, frames="pairs")
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    agent = A3C(model, opt, T, 0.99, beta=1e-2)
    pairs, rewards, dones = bench.synth_pools(N, 8, 0, dev)
    agent.run_window(pairs, rewards, dones, 8, first=True)
    for _ in range(3):
        agent.run_window(pairs, rewards, dones, 8)
    net = model.net
    for _ in range(3):
        net.run_stage("conv_bwd", 0)
    torch.cuda.synchronize()
    G = min(N * T, 256)
    raw = net.buffer("slab", torch.int32)[: G * SLAB].view(G, SLAB)[:, SLAB_W1:SLAB_W1 + 40].cpu().numpy()
    raw = raw.astype(np.int64) & 0xFFFFFFFF
    nst = raw[:, 0]
    hwid, xcc = raw[:, 1], raw[:, 2]
    t0 = raw[:, 3] | (raw[:, 4] << 32)
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 0x7
    key = list(zip(xcc & 0xF, se, sh, cu))
    start = t0 - t0.min()
    per = defaultdict(list)
    ends = []
    for b in range(G):
        st = raw[b, 8:8 + nst[b]]
        ends.append(start[b] + st[-1])
        k = len(st) - 1
        for i in range(k):
            if i == 0:
                continue
            per[PH[(i - 1) % 4]].append(st[i] - st[i - 1])
    occ = defaultdict(int)
    for k in key:
        occ[k] += 1
    print(f"workgroups {G}, CUs used {len(occ)}, workgroups per CU histogram",
          dict(sorted(defaultdict(int, {v: sum(1 for x in occ.values() if x == v) for v in set(occ.values())}).items())))
    print(f"start spread (ticks): median {np.median(start):.0f} max {start.max():.0f}; end max {max(ends):.0f}")
    nsmp = (nst - 1) // 4
    print("samples per workgroup histogram", {int(v): int((nsmp == v).sum()) for v in np.unique(nsmp)})
    for p in PH:
        v = np.array(per[p])
        print(f"{p:12s} n={len(v):5d} median {np.median(v):8.0f} mean {v.mean():8.0f} p90 {np.percentile(v, 90):8.0f} ticks")
    # same-CU pairs: do they overlap in time?
    pairs_ = defaultdict(list)
    for b in range(G):
        pairs_[key[b]].append(b)
    ov = []
    for k, bs in pairs_.items():
        if len(bs) == 2:
            a_, b_ = bs
            s0, e0 = start[a_], ends[a_]
            s1, e1 = start[b_], ends[b_]
            ov.append(max(0, min(e0, e1) - max(s0, s1)) / max(e0 - s0, e1 - s1))
    if ov:
        print(f"co-resident pairs {len(ov)}: overlap fraction median {np.median(ov):.2f} min {min(ov):.2f}")


if __name__ == "__main__":
    main()
