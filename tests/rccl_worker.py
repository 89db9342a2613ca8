"""Worker for tests/test_gpu_bench.py: a one-rank RCCL process group on the
box's GPU.  A3C(collectives=True) issues the N > 1 window's collectives (the
sectioned all-reduce around the conv backward, then clip with the norm of
the all-reduced gradient); A3C(collectives=False) is the one-rank learner
(clip norm folded into the conv reduce).  Same seeds, same pools, two
windows: actions equal, gradients and parameters equal up to the norm's
summation order."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "async-rl_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = sys.argv[1]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", device_id=dev)
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    from sim import make_pools

    G, P, T = 64, 11, 5
    pairs, rewards, dones = make_pools(np.random.default_rng(5), P, G, "uniform")
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    dp, dr, dd = t(pairs), t(rewards), t(dones)

    def agent(collectives):
        m = A3CFF(4, n_envs=G, t_max=T, seed=99, init_seed=21, frames="pairs", device=dev)
        o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
        o.add_hook(GradientClipping(0.5))        # small threshold: the clip rate is in play
        return A3C(m, o, T, 0.99, collectives=collectives)

    res = {"backend": dist.get_backend()}
    runs = {}
    for c in (True, False):
        a = agent(c)
        acts, grads = [], []
        for w in range(2):
            a.run_window(dp, dr, dd, P, first=(w == 0))
            torch.cuda.synchronize()
            acts.append(a.net.buffer("actions", torch.int32, (T + 1, G))[:T].cpu().numpy())
            grads.append(a.net.grads.cpu().numpy().astype(np.float64))
        runs[c] = (acts, grads, a.net.params.cpu().numpy().astype(np.float64))
    (a1, g1, p1), (a0, g0, p0) = runs[True], runs[False]
    res["actions_equal"] = all(bool((x == y).all()) for x, y in zip(a1, a0))
    res["grad_rel_err"] = max(float(np.abs(x - y).max() / np.abs(y).max()) for x, y in zip(g1, g0))
    res["param_rel_err"] = float(np.abs(p1 - p0).max() / np.abs(p0).max())
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
