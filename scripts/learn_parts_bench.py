"""Time each NIPS learner part alone (arl_learn_part) on a filled FF window:
    python scripts/learn_parts_bench.py [n_envs] [reps]
Environment switches (ARL_RETURNS_SPLIT=1, ARL_FC_BWD=gemm) select A/B variants."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
from asyncrl_amd import DeviceNet  # noqa: E402
from asyncrl_amd._lib import LEARN_CONV, LEARN_HEADS_DW, LEARN_RETURNS, LEARN_TRUNK  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 200
T, A = 5, 4
net = DeviceNet(0, A, N, T)
net.reset()
g = torch.Generator(device="cuda").manual_seed(0)
net.params.copy_((torch.rand(net.params.shape, device="cuda", generator=g) - 0.5) * 0.1)
probs = torch.softmax(torch.randn((T + 1, N, A), device="cuda", generator=g), -1)
net.buffer("probs", torch.float32, (T + 1, N, A)).copy_(probs)
net.buffer("logp", torch.float32, (T + 1, N, A)).copy_(probs.log())
net.buffer("v", torch.float32, (T + 1, N)).copy_(torch.randn((T + 1, N), device="cuda", generator=g))
net.buffer("rewards", torch.float32, (T, N)).copy_(torch.randn((T, N), device="cuda", generator=g))
net.buffer("hfc", torch.float32, (T + 1, N, 256)).copy_(torch.relu(torch.randn((T + 1, N, 256), device="cuda",
                                                                              generator=g)))
s = torch.cuda.current_stream()
for name, parts in (("returns", [LEARN_RETURNS]), ("heads_dw", [LEARN_HEADS_DW]), ("trunk", [LEARN_TRUNK]),
                    ("conv", [LEARN_CONV])):
    for _ in range(5):
        net.learn_parts(parts)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(REPS):
        net.learn_parts(parts)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"learn part {name} N={N} split={os.environ.get('ARL_RETURNS_SPLIT', '0')}: "
          f"{e0.elapsed_time(e1) * 1000 / REPS:.2f} us")
