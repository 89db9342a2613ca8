"""Runs two LSTM windows (eager + graph-captured) and one pi_and_v call and
saves actions, values, hidden states, gradients and parameters to an .npz
(argv[1]); test_gpu_parity.test_lstm_fc_reduce_forms_identical runs it under
ARL_LSTM_XRED and compares the files bitwise.  argv[2] == "one": a single window,
its gradients (flat and per tensor) and dfc only."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "async-rl_amd"), os.path.join(HERE, "..", "oracle"), HERE]
from sim import make_pools  # noqa: E402
from asyncrl_amd import A3C, A3CLSTM, GradientClipping, RMSpropAsync  # noqa: E402


def main(out, one=False):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(123)
    N, T, P = int(os.environ.get("LSTM_WORKER_N", "72")), 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.15)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    dp, dr, dd = t(pairs), t(rewards), t(dones)
    m = A3CLSTM(6, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs", device=dev)
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
    o.add_hook(GradientClipping(40))
    ag = A3C(m, o, T, 0.99)
    ag.run_window(dp, dr, dd, P, first=True, env_groups=2, split_update=one)
    if one:
        torch.cuda.synchronize()
        per = {"g." + k.replace("/", "."): np.asarray(v.detach().cpu().numpy() if torch.is_tensor(v) else v)
               for k, v in ag.net.state_dict(ag.net.grads).items()}
        np.savez(out, grads=ag.net.grads.detach().cpu().numpy(),
                 hbuf=ag.net.buffer("hbuf", torch.float32).detach().cpu().numpy(),
                 dfc=ag.net.buffer("dfc", torch.float32).detach().cpu().numpy(), **per)
        return
    ag.run_window(dp, dr, dd, P, env_groups=1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ag.run_window(dp, dr, dd, P, stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ag.run_window(dp, dr, dd, P, stream=s, split_update=True)
    g.replay()
    torch.cuda.synchronize()
    net = ag.net
    x = torch.rand((N, 4, 84, 84), generator=torch.Generator().manual_seed(3)).to(dev)
    pout, v = m.pi_and_v(x, deterministic=True)
    res = {"actions": net.buffer("actions", torch.int32, (T + 1, N)), "v": net.buffer("v", torch.float32, (T + 1, N)),
           "hbuf": net.buffer("hbuf", torch.float32), "cbuf": net.buffer("cbuf", torch.float32),
           "gates": net.buffer("gates", torch.float32), "grads": net.grads, "params": net.params, "ms": net.ms,
           "eval_v": v, "eval_probs": pout.probs}
    np.savez(out, **{k: r.detach().cpu().numpy() for k, r in res.items()})


if __name__ == "__main__":
    main(sys.argv[1], len(sys.argv) > 2 and sys.argv[2] == "one")
