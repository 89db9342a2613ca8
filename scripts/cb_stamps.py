"""Per-phase timeline of conv_bwd_kernel from an ARL_CB_STAMP build
(make -C async-rl_amd/csrc variant NAME=cbstamp DEFS="-DARL_CB_STAMP=1"):
s_memtime at every barrier of the sample loop, written into each workgroup's
slab (the gradients are wrong by design).
    ASYNCRL_HIP_LIB=.../build_var_cbstamp/libasyncrl_hip.so python scripts/cb_stamps.py [n_envs]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "async-rl_amd")]
import bench  # noqa: E402
from asyncrl_amd import A3C, A3CFF, RMSpropAsync  # noqa: E402

SLAB_W1, SLAB = 8224, 12336
PH = ["commit (+ a1 DMA wait)", "(1) conv2 dW + mask", "(2) convT da1", "(3) conv1 dW"]


def main():
    dev = torch.device("cuda", 0)
    N, T = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 5
    model = A3CFF(4, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev, frames="pairs")
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    agent = A3C(model, opt, T, 0.99, beta=1e-2)
    pairs, rewards, dones = bench.synth_pools(N, 8, 0, dev)
    agent.run_window(pairs, rewards, dones, 8, first=True)
    net = model.net
    for _ in range(3):
        net.run_stage("conv_bwd", 0)
    torch.cuda.synchronize()
    G = min(256, N * T)
    sl = net.buffer("slab", torch.float32, None)[:G * SLAB].view(G, SLAB).view(torch.int32).cpu().numpy()
    o = sl[:, SLAB_W1:].astype(np.int64) & 0xffffffff
    nst = o[:, 0]
    n = int(nst.min())
    print(f"N = {N}: {G} workgroups, stamps per workgroup {n}..{int(nst.max())} (kept <= 30)")
    st = o[:, 8:8 + min(n, 30)].astype(np.float64)
    d = np.diff(st, axis=1)
    # stamp 4 j + k: sample j past barrier B0 / B1 / B2 / B3; the interval after stamp 4 j + k is phase k
    for k in range(4):
        cols = [4 * j + k for j in range(d.shape[1] // 4 + 1) if 4 * j + k < d.shape[1]]
        v = d[:, cols]
        print(f"{PH[k]:24s} median {np.median(v):8.0f}  mean {v.mean():8.0f} ticks  ({len(cols)} samples a wg)")
    per = d[:, :4 * (d.shape[1] // 4)].reshape(G, -1, 4).sum(2)
    print(f"per sample: median {np.median(per):.0f} ticks; first stamp median {np.median(st[:, 0]):.0f}")


if __name__ == "__main__":
    main()
