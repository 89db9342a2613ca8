"""Runs two FF windows (the second graph-captured) at argv[2] envs with one
env group and saves a1, a2, the actions, the window-1 gradient and the
parameters to an .npz (argv[1]).  test_gpu_parity.test_conv_fwd_two_envs_identical
runs it under ARL_CONV_EPW=1 / 2 (conv_fwd.hip: one or two envs a workgroup,
read once per process), ARL_FC_BIG and ARL_WINDOW_C and compares the files bitwise."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "async-rl_amd"), os.path.join(HERE, "..", "oracle"), HERE]
from sim import make_pools  # noqa: E402
from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync  # noqa: E402


def main(out, N):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(77)
    T, P = 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    dp, dr, dd = t(pairs), t(rewards), t(dones)
    m = A3CFF(4, n_envs=N, t_max=T, seed=9, init_seed=10, frames="pairs", device=dev)
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
    o.add_hook(GradientClipping(40))
    ag = A3C(m, o, T, 0.99)
    ag.run_window(dp, dr, dd, P, first=True, env_groups=1)
    torch.cuda.synchronize()
    g1 = ag.net.grads.detach().cpu().numpy().copy()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ag.run_window(dp, dr, dd, P, stream=s, env_groups=1)
    g.replay()
    torch.cuda.synchronize()
    net = ag.net
    np.savez(out, grads1=g1, params=net.params.detach().cpu().numpy(),
             a1=net.buffer("a1", torch.float32).cpu().numpy(), a2=net.buffer("a2", torch.float32).cpu().numpy(),
             frames=net.buffer("frames").cpu().numpy(),
             actions=net.buffer("actions", torch.int32, (T + 1, N)).cpu().numpy(),
             **{k: net.buffer(k, torch.float32).cpu().numpy() for k in ("hfc", "logits", "probs", "logp", "v",
                                                                       "entropy", "logp_a", "dlogits", "dv",
                                                                       "loss", "dfc")})


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
