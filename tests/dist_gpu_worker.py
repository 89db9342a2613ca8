"""Worker for tests/test_gpu_dist.py: 2 ranks on ONE GPU (gloo transport;
RCCL needs one GPU per rank), env-sharded A3C over 2 windows.  Rank 0 also
runs the single-process learner over the union of envs for comparison."""
import json
from datetime import timedelta
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "async-rl_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync  # noqa: E402
from asyncrl_amd.distributed import replicas_identical, shard_envs  # noqa: E402
from sim import make_pools  # noqa: E402


def agent(n, off, group):
    m = A3CFF(4, n_envs=n, t_max=5, seed=99, env_offset=off, init_seed=21, frames="pairs")
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
    o.add_hook(GradientClipping(40))
    return A3C(m, o, 5, 0.99, process_group=group)


def main():
    out = sys.argv[1]
    dist.init_process_group("gloo", timeout=timedelta(seconds=240))
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    G, P = 8, 11
    pairs, rewards, dones = make_pools(np.random.default_rng(3), P, G, "uniform")
    n, off = shard_envs(G, world, rank)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    dp, dr, dd = t(pairs[:, off:off + n]), t(rewards[:, off:off + n]), t(dones[:, off:off + n])
    solo_group = dist.new_group([0])
    a = agent(n, off, None)
    same = []
    acts0 = None
    for w in range(2):
        a.run_window(dp, dr, dd, P, first=(w == 0))
        torch.cuda.synchronize()
        if w == 0:
            acts0 = a.net.buffer("actions", torch.int32, (6, n))[:5].cpu().numpy()
        same.append(replicas_identical(a.net.params) and replicas_identical(a.net.ms))
    res = {"rank": rank, "identical": same}
    acts = [torch.zeros((5, n), dtype=torch.int32) for _ in range(world)]
    dist.all_gather(acts, torch.from_numpy(acts0))
    if rank == 0:
        s = agent(G, 0, solo_group)
        p0 = s.net.params.clone()
        ap, ar, ad = t(pairs), t(rewards), t(dones)
        for w in range(2):
            s.run_window(ap, ar, ad, P, first=(w == 0))
            torch.cuda.synchronize()
            if w == 0:
                sacts = s.net.buffer("actions", torch.int32, (6, G))[:5].cpu().numpy()
        d_sh = (a.net.params - p0).cpu().numpy().astype(np.float64)
        d_so = (s.net.params - p0).cpu().numpy().astype(np.float64)
        scale = np.maximum(np.abs(d_so), np.abs(d_so).max())
        res["delta_rel_err"] = float((np.abs(d_sh - d_so) / scale).max())
        res["actions_equal"] = bool((np.concatenate([x.numpy() for x in acts], 1) == sacts).all())
        with open(out, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
