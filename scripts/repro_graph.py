"""Capture + replay one window graph: python scripts/repro_graph.py <arch> <N> <groups> [first_eager_windows]
(diagnostic for graph captures that mix env-group streams with the learner's side stream)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
sys.path.insert(0, ROOT)

from asyncrl_amd import A3C, A3CFF, A3CLSTM, GradientClipping, RMSpropAsync  # noqa: E402
from bench import synth_pools  # noqa: E402

arch, N, G = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
dev = torch.device("cuda", 0)
T, P = 5, 4
Model = {"ff": A3CFF, "lstm": A3CLSTM}[arch]
m = Model(4, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev)
o = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(m)
o.add_hook(GradientClipping(40))
ag = A3C(m, o, T, 0.99)
pairs, rewards, dones = synth_pools(N, P, 0, dev)
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    ag.run_window(pairs, rewards, dones, P, first=True, stream=s, env_groups=G)
    ag.run_window(pairs, rewards, dones, P, stream=s, env_groups=G)
s.synchronize()
print("eager ok", flush=True)
g = torch.cuda.CUDAGraph()
split = len(sys.argv) > 4 and sys.argv[4] == "split"
with torch.cuda.graph(g, stream=s):
    ag.run_window(pairs, rewards, dones, P, stream=s, env_groups=G, split_update=split)
print("captured", flush=True)
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", i, "ok", flush=True)
print("finite", bool(torch.isfinite(m.net.params).all()))
