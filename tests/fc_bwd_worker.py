"""Runs FF windows at 256 envs (S = 1,280 samples: two FC-backward dW ranges)
and saves the window-1 gradient, the parameters after three windows and the
actions to an .npz (argv[1]).  test_gpu_parity.test_fc_bwd_variants runs it
under the FC backward's build-free knobs (ARL_FC_BWD_SPIN, ARL_FC_BWD_F32,
read once per process) and compares the files."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "async-rl_amd"), os.path.join(HERE, "..", "oracle"), HERE]
from sim import make_pools  # noqa: E402
from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync  # noqa: E402


def main(out):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(321)
    N, T, P = 256, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    dp, dr, dd = t(pairs), t(rewards), t(dones)
    m = A3CFF(4, n_envs=N, t_max=T, seed=7, init_seed=8, frames="pairs", device=dev)
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
    o.add_hook(GradientClipping(40))
    ag = A3C(m, o, T, 0.99)
    ag.run_window(dp, dr, dd, P, first=True)
    torch.cuda.synchronize()
    g1 = ag.net.grads.detach().cpu().numpy().copy()
    ag.run_window(dp, dr, dd, P)
    ag.run_window(dp, dr, dd, P)
    torch.cuda.synchronize()
    net = ag.net
    np.savez(out, grads1=g1, params=net.params.detach().cpu().numpy(),
             actions=net.buffer("actions", torch.int32, (T + 1, N)).cpu().numpy())


if __name__ == "__main__":
    main(sys.argv[1])
