"""Per-phase timeline of conv_fwd_kernel<false> from an ARL_CF_STAMP build
(make -C async-rl_amd/csrc variant NAME=cfstamp DEFS="-DARL_CF_STAMP=1"):
s_memtime at the phase ends, written into a2 (results wrong by design).
    ASYNCRL_HIP_LIB=.../build_var_cfstamp/libasyncrl_hip.so python scripts/cf_stamps.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "async-rl_amd")]
import bench  # noqa: E402
from asyncrl_amd import A3C, A3CFF, RMSpropAsync  # noqa: E402

PH = ["staged", "barrier", "conv1 (+ barrier)", "a1 epilogue", "barrier", "W2 frags", "conv2", "end"]


def main():
    dev = torch.device("cuda", 0)
    N, T = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 5   # 512: conv_fwd_kernel<false, 2> (two envs a workgroup)
    model = A3CFF(4, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev, frames="pairs")
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    agent = A3C(model, opt, T, 0.99, beta=1e-2)
    pairs, rewards, dones = bench.synth_pools(N, 8, 0, dev)
    agent.run_window(pairs, rewards, dones, 8, first=True)
    net = model.net
    for _ in range(3):
        net.run_stage("conv_fwd", 2)
    torch.cuda.synchronize()
    a2 = net.buffer("a2", torch.float32, (T + 1, N, 2592))[2].contiguous().view(torch.int32).cpu().numpy()
    st = a2[:, :80].reshape(N, 8, 10).astype(np.int64) & 0xffffffff
    t0 = st[:, 0, 8] + (st[:, 0, 9] << 32)
    print(f"N = {N}: start spread (ticks): max - min", int(t0.max() - t0.min()))
    prev = np.zeros((N, 8))
    for k, name in enumerate(PH):
        v = st[:, :, k].astype(np.float64)
        d = v - prev
        prev = v
        print(f"{k} {name:12s} at {np.median(v):8.0f}  delta median {np.median(d):7.0f}  max-wave {np.median(d.max(1)):7.0f}")


if __name__ == "__main__":
    main()
