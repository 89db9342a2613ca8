"""Diagnose per-element FC weight-gradient differences (device vs oracle):
runs one FF window at N envs, then for the worst elements of 0/2/W (in
units of the oracle's summand scale) splits the difference into the GEMM
itself (device dW vs sum of the device's own dfc x a2) and its operands."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "async-rl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O  # noqa: E402
from sim import OracleEnvView, make_pools  # noqa: E402
from asyncrl_amd import A3C, A3CFF, RMSpropAsync  # noqa: E402

gpu = torch.device("cuda:0")
N, T, A, seed = int(sys.argv[1]) if len(sys.argv) > 1 else 6, 5, 4, 21
rng = np.random.default_rng(seed)
P = 2 * T + 1
pairs, rewards, dones = make_pools(rng, P, N, "uniform")
model = A3CFF(A, n_envs=N, t_max=T, seed=99, init_seed=seed, frames="pairs")
agent = A3C(model, RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(model), T, 0.99)
net = model.net
view = OracleEnvView(pairs, dones)
dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(gpu)  # noqa: E731
params = net.state_dict()
agent.run_window(dev(pairs), dev(rewards), dev(dones), P, first=True, split_update=True)
torch.cuda.synchronize()
states, boot = view.states_f32(0, T)
r, d = view.window_rd(rewards, 0, T)
acts = net.buffer("actions", torch.int32, (T + 1, N))[:T].cpu().numpy()
da = (net.buffer("a1", torch.float32, (T + 1, N, 16, 20, 20))[:T].cpu().numpy().reshape(T * N, 16, 20, 20),
      net.buffer("a2", torch.float32, (T + 1, N, 32, 9, 9))[:T].cpu().numpy().reshape(T * N, 32, 9, 9),
      net.buffer("hfc", torch.float32, (T + 1, N, 256))[:T].cpu().numpy().reshape(T * N, 256))
g, aux = O.ff_window_grads(params, states, acts, r, d, boot, dev_acts=da)
got = net.state_dict(net.grads)["0/2/W"]
want = g["0/2/W"]
mag = aux["grad_mag"]["0/2/W"]
err = np.abs(got - want) / np.maximum(mag, 1e-7 * mag.max())
dfc_dev = net.buffer("dfc", torch.float32, (T * N, 256)).cpu().numpy()
a2_dev = da[1].reshape(T * N, -1)
# oracle's own operands
x = states.reshape(T * N, 4, 84, 84)
a1o, a2o, ho = O.nips_head(params, O.ARCH_FF, x)
a2o = a2o.reshape(T * N, -1)
dl = aux["dlogits"].reshape(T * N, A)
dv = aux["dv"].reshape(T * N)
dho = dl @ params["1/0/W"] + dv[:, None] * params["2/0/W"]
dfco = dho * O.relu_mask(ho, da[2])
print("max err (units of mag)", err.max(), "count > 1e-3:", int((err > 1e-3).sum()))
print("dfc dev vs oracle: max abs", np.abs(dfc_dev - dfco).max(), "max |dfc|", np.abs(dfco).max())
print("a2 dev vs oracle: max abs", np.abs(a2_dev - a2o).max(), "max |a2|", np.abs(a2o).max())
dl_dev = net.buffer("dlogits", torch.float32, (T, N, A)).cpu().numpy().reshape(T * N, A)
print("dlogits dev vs oracle: max abs", np.abs(dl_dev - dl).max(), "max", np.abs(dl).max())
for flat in np.argsort(err.ravel())[::-1][:5]:
    j, k = np.unravel_index(flat, err.shape)
    own = float((dfc_dev[:, j].astype(np.float64) * a2_dev[:, k]).sum())
    ora = float((dfco[:, j].astype(np.float64) * a2o[:, k]).sum())
    print(f"({j},{k}) dev {got[j, k]:.9g} oracle {want[j, k]:.9g} mag {mag[j, k]:.3g} err {err[j, k]:.3g} | "
          f"sum(dev ops) {own:.9g} sum(oracle ops) {ora:.9g}")
    terms = dfco[:, j] * a2o[:, k]
    idx = np.argsort(-np.abs(terms))[:4]
    for s in idx:
        print(f"     s={s} dfc dev {dfc_dev[s, j]:.9g} ora {dfco[s, j]:.9g}  a2 dev {a2_dev[s, k]:.9g} ora {a2o[s, k]:.9g}")
