"""Phase stamps of conv_bwd_ws_kernel (diagnostic): run C4 windows (512 envs, T = 5) on the stamp build
(async-rl_amd/csrc/build_var_wsstamp, make variant NAME=wsstamp DEFS=-DARL_CB_WS_STAMP) with ARL_CB_WS=1 and
print, per sample k, the P / Q phase lengths and each wave group's busy part (shader clocks, median over
workgroups 0-7 of the last window)."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.environ.get("VAR", "wsstamp")
sys.path.insert(0, os.path.join(ROOT, "async-rl_amd", "csrc", "build_var_" + VAR))
sys.path.insert(0, ROOT)
os.environ.setdefault("ARL_CB_WS", "1")
import torch  # noqa: E402

import asyncrl_amd  # noqa: E402
from asyncrl_amd import _lib  # noqa: E402
from bench import synth_pools  # noqa: E402

assert "build_var_" + VAR in _lib.LIB_PATH, _lib.LIB_PATH
dev = torch.device("cuda", 0)
N, T, P = int(os.environ.get("N", "512")), 5, 8
m = asyncrl_amd.A3CFF(4, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev, frames="pairs")
o = asyncrl_amd.RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
o.add_hook(asyncrl_amd.GradientClipping(40))
ag = asyncrl_amd.A3C(m, o, T, 0.99)
pairs, rewards, dones = synth_pools(N, P, 0, dev)
for i in range(6):
    ag.run_window(pairs, rewards, dones, P, first=(i == 0))
torch.cuda.synchronize()
buf = np.zeros((8, 2, 16, 6), np.uint64)
f = _lib.lib.arl_debug_cb_stamps
f.argtypes = [ctypes.c_void_p]
assert f(buf.ctypes.data) == 0
st = buf.astype(np.int64)
S = N * T
n = (S - 1) // min(S, 256) + 1
X, Y = st[:, 0], st[:, 1]
rows = []
for k in range(min(n, 15)):
    p_len = (X[:, k, 2] - X[:, k, 0]) if True else None
    q_end = X[:, k + 1, 0] if k + 1 < min(n, 15) else X[:, k, 3]
    rows.append({"k": k, "P": int(np.median(p_len)), "X_P_work": int(np.median(X[:, k, 1] - X[:, k, 0])),
                 "Y_P_work": int(np.median(Y[:, k, 1] - Y[:, k, 0])), "Q": int(np.median(q_end - X[:, k, 2])),
                 "X_Q_work": int(np.median(X[:, k, 3] - X[:, k, 2])), "Y_Q_work": int(np.median(Y[:, k, 3] - Y[:, k, 2])),
                 "Y_S1_end": int(np.median(Y[:, k, 4] - Y[:, k, 0])), "Y_slot5": int(np.median(Y[:, k, 5] - Y[:, k, 0]))})
pro = {"to_b1": int(np.median(X[:, 15, 1] - X[:, 15, 0])), "fill_b2": int(np.median(X[:, 15, 2] - X[:, 15, 1])),
       "b3": int(np.median(X[:, 15, 3] - X[:, 15, 2])),
       "Y_issue": int(np.median(Y[:, 15, 1] - Y[:, 15, 0])), "Y_wait": int(np.median(Y[:, 15, 2] - Y[:, 15, 1])),
       "Y_commit": int(np.median(Y[:, 15, 3] - Y[:, 15, 2])), "Y_start_minus_X_start": int(np.median(Y[:, 15, 0] - X[:, 15, 0]))}
total = int(np.median(X[:, n - 1 if n < 15 else 14, 3] - X[:, 15, 0]))
print(json.dumps({"N": N, "samples_per_wg": n, "prologue": pro, "total_clocks": total}))
for r in rows:
    print(json.dumps(r))
