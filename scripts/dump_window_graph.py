"""Dump the captured window graph (torch.cuda.CUDAGraph debug dump, .dot) for
a given env-group count, to inspect its branch structure:
    python scripts/dump_window_graph.py 2 gpurun_out/window_g2.dot
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
sys.path.insert(0, ROOT)

from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync  # noqa: E402
from bench import synth_pools  # noqa: E402

groups, out = int(sys.argv[1]), sys.argv[2]
dev = torch.device("cuda", 0)
N, T, P = 256, 5, 4
model = A3CFF(4, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev)
opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
opt.add_hook(GradientClipping(40))
agent = A3C(model, opt, T, 0.99)
pairs, rewards, dones = synth_pools(N, P, 0, dev)
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    agent.run_window(pairs, rewards, dones, P, first=True, stream=s, env_groups=groups)
    agent.run_window(pairs, rewards, dones, P, stream=s, env_groups=groups)
s.synchronize()
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
with torch.cuda.graph(g, stream=s):
    agent.run_window(pairs, rewards, dones, P, stream=s, env_groups=groups)
g.debug_dump(out)
print("dumped", out)
