"""FC backward stage alone (arl_run_stage fc_bwd) on random window data:
average launch time over many back-to-back launches between HIP events.
    python scripts/fc_bwd_bench.py [n_envs] [reps] [arch ff|lstm]
ARL_FC_BWD=gemm selects the round-1 GEMM pair + reduce, ARL_FC_BWD_JOBS=a|b
one job of fc_bwd_kernel alone."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
from asyncrl_amd import DeviceNet  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
arch = 1 if (len(sys.argv) > 3 and sys.argv[3] == "lstm") else 0
T = 5
net = DeviceNet(arch, 4, N, T)
net.reset()
g = torch.Generator(device="cuda").manual_seed(0)
net.params.copy_(torch.rand(net.params.shape, device="cuda", generator=g) - 0.5)
for name, shape in (("a2", ((T + 1) * N, 2592)), ("dfc", (T * N, 256))):
    b = net.buffer(name, torch.float32, shape)
    b.copy_(torch.relu(torch.randn(shape, device="cuda", generator=g)))
s = torch.cuda.current_stream()
for _ in range(10):
    net.run_stage("fc_bwd")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(REPS):
    net.run_stage("fc_bwd")
e1.record(s)
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / REPS
flop = 2 * 2 * T * N * 256 * 2592
print(f"fc_bwd N={N} S={T * N} variant={os.environ.get('ARL_FC_BWD', 'fc_bwd_kernel')} "
      f"jobs={os.environ.get('ARL_FC_BWD_JOBS', 'ab')}: {us:.2f} us/launch, {flop / us / 1e6:.1f} TFLOP/s")
