"""Per-phase timeline of fc_fwd_kernel from a stamped build (an experiment
build, never the product: lane 0 of every wave writes s_memtime at kernel
start, after each of the 4 chunk waits, after each chunk's MFMAs and after
the partial stores, 10 u64 a wave, into the FC slab past its partials).
    ASYNCRL_HIP_LIB=.../build_var_fcst/libasyncrl_hip.so python scripts/fc_stamps.py [N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "async-rl_amd")]
import bench  # noqa: E402
from asyncrl_amd import A3C, A3CFF, RMSpropAsync  # noqa: E402

PH = ["start", "chunk0 landed", "chunk1 landed", "chunk2 landed", "chunk3 landed",
      "chunk0 mfma", "chunk1 mfma", "chunk2 mfma", "chunk3 mfma", "partials stored"]
ORDER = [0, 1, 5, 2, 6, 3, 7, 4, 8, 9]


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
        net.run_stage("fc_fwd", 2)
    torch.cuda.synchronize()
    big = N >= 512
    nw = 16 if big else 8
    wg = (-(-N // (64 if big else 32))) * 4 * 8
    slab = net.buffer("slab", torch.float32)
    base = 8 * N * 256
    st = slab[base:base + wg * nw * 20].view(torch.int64).cpu().numpy().reshape(wg, nw, 10).astype(np.float64)
    t0 = st[:, :, 0].min()
    st -= t0
    print(f"N = {N}: {wg} workgroups x {nw} waves; s_memtime ticks from the first wave's start")
    print(f"  start spread: wg start min {st[:, :, 0].min(1).min():.0f} median {np.median(st[:, :, 0].min(1)):.0f} "
          f"max {st[:, :, 0].min(1).max():.0f}")
    prev = st[:, :, 0]
    for k in ORDER:
        v = st[:, :, k]
        d = v - prev
        prev = v
        print(f"  {PH[k]:16s} at median {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f}   "
              f"delta median {np.median(d):7.0f} p90 {np.percentile(d, 90):7.0f}")
    print(f"  end of last wave {st[:, :, 9].max():.0f}")


if __name__ == "__main__":
    main()
