"""Generate the golden fixtures under tests/golden/ from the reference's OWN code.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/gen_golden.py

What runs from the reference (nothing is copied; modules are imported from
/root/reference at generation time only):
  * dqn_phi.dqn_phi                -- imported directly (numpy only).
  * ale.ALE.current_screen / initialize / receive_action / state
                                   -- imported with two stub modules for
    absent third-party packages: `ale_python_interface` (a fake emulator that
    serves seeded synthetic 210x160x3 frames, lives and rewards) and `cv2`
    (its `resize` records the reference's luminance image and answers with
    the oracle's OpenCV restatement, so resize parity stays "unpinned").
  * rmsprop_async.RMSpropAsync.update_one_cpu
                                   -- imported with a minimal `chainer` stub
    (`cuda.get_array_module`, `optimizer.GradientMethod`), run on NumPy arrays.
  * trained_model/breakout_ff/80000000_finish.h5
                                   -- read with h5py (conda python3.9; plain
    HDF5 datasets, nothing executed) and saved as breakout_ff.npz.

Outputs are data only (inputs + expected outputs).
"""
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))
import oracle  # noqa: E402
from fake_ale import FakeALE, synth_frames  # noqa: E402  (tests/fake_ale.py)


# --------------------------------------------------------------------------
# stubs for absent third-party modules
# --------------------------------------------------------------------------
RESIZE_LOG = []


def _resize_rows(img, dst_h):
    """84-column, dst_h-row restatement of the OpenCV resize (the oracle's
    passes with the 210 -> dst_h row coefficients) for the cv2 stub."""
    ys, yb = oracle.resize_coeffs(oracle.SRC_H, dst_h)
    src = img.astype(np.int64)
    xs, xa = oracle.resize_coeffs(oracle.SRC_W, oracle.DST)
    rows = src[:, xs] * xa[:, 0] + src[:, np.minimum(xs + 1, oracle.SRC_W - 1)] * xa[:, 1]
    r0, r1 = rows[ys, :], rows[np.minimum(ys + 1, oracle.SRC_H - 1), :]
    out = (yb[:, 0][:, None] * r0 + yb[:, 1][:, None] * r1 + (1 << 21)) >> 22
    return np.clip(out, 0, 255).astype(np.uint8)


def install_cv2_stub():
    cv2 = types.ModuleType("cv2")
    cv2.INTER_LINEAR = 1

    def resize(img, dsize, interpolation=None):
        assert dsize in ((84, 84), (84, 110)) and interpolation == 1
        RESIZE_LOG.append(np.array(img, copy=True))
        if dsize == (84, 110):          # ale.py:75-76, the 'crop' branch
            return _resize_rows(img, 110)
        return oracle.resize_linear_u8(img, oracle.RESIZE_SCALAR)

    cv2.resize = resize
    sys.modules["cv2"] = cv2


def install_ale_stub():
    m = types.ModuleType("ale_python_interface")
    m.ALEInterface = FakeALE
    sys.modules["ale_python_interface"] = m


def install_chainer_stub():
    ch = types.ModuleType("chainer")
    cuda = types.ModuleType("chainer.cuda")
    cuda.get_array_module = lambda *a: np
    opt = types.ModuleType("chainer.optimizer")

    class GradientMethod(object):
        pass

    opt.GradientMethod = GradientMethod
    ch.cuda = cuda
    ch.optimizer = opt
    sys.modules["chainer"] = ch
    sys.modules["chainer.cuda"] = cuda
    sys.modules["chainer.optimizer"] = opt


# --------------------------------------------------------------------------
def gen_phi():
    rng = np.random.default_rng(1)
    cur, prev = [], []
    for kind, n in (("uniform", 2), ("palette", 2), ("white", 1), ("black", 1)):
        cur.append(synth_frames(rng, n, kind))
        prev.append(synth_frames(rng, n, kind))
    # one pair mixing white and uniform so max() matters
    cur.append(synth_frames(rng, 1, "white"))
    prev.append(synth_frames(rng, 1, "uniform"))
    cur = np.concatenate(cur)
    prev = np.concatenate(prev)

    install_cv2_stub()
    install_ale_stub()
    sys.path.insert(0, REF)
    import ale  # reference ale.py

    gray = []
    shots = []
    for i in range(cur.shape[0]):
        env = ale.ALE.__new__(ale.ALE)
        env.crop_or_scale = "scale"
        env.ale = types.SimpleNamespace(getScreenRGB=lambda i=i: cur[i])
        env.last_raw_screen = prev[i]
        RESIZE_LOG.clear()
        shots.append(env.current_screen())          # ale.py:59-89 verbatim
        gray.append(RESIZE_LOG[0])
    gray = np.stack(gray)
    np.savez_compressed(os.path.join(HERE, "phi_golden.npz"), cur=cur, prev=prev,
                        gray=gray, screen_scalar=np.stack(shots))

    # ---- episode stack semantics through ALE.initialize / receive_action
    np.random.seed(5)
    fake_pairs = []
    orig_cs = ale.ALE.current_screen

    def logged_cs(self):
        fake_pairs.append((self.ale.getScreenRGB().copy(), self.last_raw_screen.copy()))
        return orig_cs(self)

    ale.ALE.current_screen = logged_cs
    env = ale.ALE("fake.rom", seed=3, max_start_nullops=4)
    states, terms, pair_idx = [np.array(env.state)], [False], [len(fake_pairs) - 1]
    resets = [True]
    for step in range(24):
        if env.is_terminal:
            env.initialize()
            resets.append(True)
        else:
            env.receive_action(step % 4)
            resets.append(False)
        states.append(np.array(env.state))
        terms.append(bool(env.is_terminal))
        pair_idx.append(len(fake_pairs) - 1)
    ale.ALE.current_screen = orig_cs
    cur_f = np.stack([p[0] for p in fake_pairs])
    prev_f = np.stack([p[1] for p in fake_pairs])
    np.savez_compressed(os.path.join(HERE, "ale_stack_golden.npz"),
                        pair_cur=cur_f, pair_prev=prev_f,
                        states=np.stack(states), terminal=np.array(terms),
                        reset=np.array(resets), pair_idx=np.array(pair_idx))
    sys.path.remove(REF)


def gen_phi_crop():
    """ale.py:73-82 (crop_or_scale='crop') run verbatim on the phi_golden
    frame pairs: pins the crop window (rows 18..101 of the 84 x 110 resize);
    the resize itself is the stub's restatement (unpinned, as for 'scale')."""
    install_cv2_stub()
    install_ale_stub()
    sys.path.insert(0, REF)
    import ale  # reference ale.py
    d = np.load(os.path.join(HERE, "phi_golden.npz"))
    shots = []
    for i in range(d["cur"].shape[0]):
        env = ale.ALE.__new__(ale.ALE)
        env.crop_or_scale = "crop"
        env.ale = types.SimpleNamespace(getScreenRGB=lambda i=i: d["cur"][i])
        env.last_raw_screen = d["prev"][i]
        shots.append(env.current_screen())
    np.savez_compressed(os.path.join(HERE, "phi_crop_golden.npz"), screen_crop=np.stack(shots))
    sys.path.remove(REF)


def gen_ale_env():
    """ale.ALE (ale.py:11-161) driven like a3c_ale.py's train loop over an
    action-sensitive fake emulator: per receive_action the action, reward,
    terminal flag and the raw frame pair behind the next observation (the
    pair of the following initialize() when the step was terminal)."""
    import fake_ale
    install_cv2_stub()
    m = types.ModuleType("ale_python_interface")
    m.ALEInterface = fake_ale.FakeALEActions
    sys.modules["ale_python_interface"] = m
    sys.path.insert(0, REF)
    for k in [k for k in sys.modules if k == "ale"]:
        del sys.modules[k]
    import ale  # reference ale.py
    pairs = []
    orig_cs = ale.ALE.current_screen

    def logged_cs(self):
        pairs.append((self.ale.getScreenRGB().copy(), self.last_raw_screen.copy()))
        return orig_cs(self)

    ale.ALE.current_screen = logged_cs
    np.random.seed(7)
    env = ale.ALE("fake.rom", seed=3, max_start_nullops=6)
    actions = np.random.default_rng(8).integers(0, 4, 48)
    rewards, dones, idx = [], [], [len(pairs) - 1]
    for a in actions:
        r = env.receive_action(int(a))
        term = bool(env.is_terminal)
        if term:
            env.initialize()
        rewards.append(r)
        dones.append(term)
        idx.append(len(pairs) - 1)
    ale.ALE.current_screen = orig_cs
    sel = [pairs[i] for i in idx]
    np.savez_compressed(os.path.join(HERE, "ale_env_golden.npz"), actions=actions,
                        rewards=np.array(rewards, np.float32), dones=np.array(dones),
                        pair_cur=np.stack([p[0] for p in sel]), pair_prev=np.stack([p[1] for p in sel]),
                        emulator_actions=np.array(env.ale.actions))
    sys.path.remove(REF)
    del sys.modules["ale"]
    sys.modules["ale_python_interface"].ALEInterface = FakeALE


def gen_dqn_phi():
    sys.path.insert(0, REF)
    import dqn_phi  # reference dqn_phi.py, imported directly
    rng = np.random.default_rng(2)
    stacks = rng.integers(0, 256, (3, 4, 84, 84), dtype=np.uint8)
    stacks[0, 0] = np.arange(84 * 84, dtype=np.int64).reshape(84, 84) % 256
    stacks[1, 2] = 255
    out = np.stack([dqn_phi.dqn_phi([s for s in st]) for st in stacks])
    np.savez_compressed(os.path.join(HERE, "dqn_phi_golden.npz"), stacks=stacks, out=out)
    sys.path.remove(REF)


def gen_rmsprop():
    install_chainer_stub()
    sys.path.insert(0, REF)
    import rmsprop_async  # reference rmsprop_async.py
    rng = np.random.default_rng(3)
    n = 4096
    p = rng.standard_normal(n).astype(np.float32) * 0.05
    ms = np.abs(rng.standard_normal(n)).astype(np.float32) * 0.01
    ms[:16] = 0.0
    g = rng.standard_normal(n).astype(np.float32) * 0.3
    g[16:32] = 0.0
    steps = []
    opt = rmsprop_async.RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99)
    cur_p, cur_ms = p.copy(), ms.copy()
    for k in range(3):
        # a3c_ale.py:111-112 anneal, total 8e7 steps, at global_t = 10**6*k
        opt.lr = (8 * 10 ** 7 - 10 ** 6 * k - 1) / (8 * 10 ** 7) * 7e-4
        gk = (g * (1.0 + 0.5 * k)).astype(np.float32)
        param = types.SimpleNamespace(data=cur_p.copy(), grad=gk)
        state = {"ms": cur_ms.copy()}
        opt.update_one_cpu(param, state)          # rmsprop_async.py:23-29
        steps.append((cur_p.copy(), cur_ms.copy(), gk, opt.lr, param.data.copy(),
                      state["ms"].copy()))
        cur_p, cur_ms = param.data, state["ms"]
    np.savez_compressed(
        os.path.join(HERE, "rmsprop_golden.npz"),
        p=np.stack([s[0] for s in steps]), ms=np.stack([s[1] for s in steps]),
        g=np.stack([s[2] for s in steps]), lr=np.array([s[3] for s in steps]),
        p_out=np.stack([s[4] for s in steps]), ms_out=np.stack([s[5] for s in steps]))
    sys.path.remove(REF)


def gen_checkpoint():
    src = os.path.join(REF, "trained_model/breakout_ff/80000000_finish.h5")
    dst = os.path.join(HERE, "breakout_ff.npz")
    code = ("import h5py, numpy as np, sys\n"
            "f = h5py.File(sys.argv[1], 'r')\n"
            "d = {}\n"
            "f.visititems(lambda n, o: d.__setitem__(n, o[()]) "
            "if isinstance(o, h5py.Dataset) else None)\n"
            "np.savez_compressed(sys.argv[2], **{k.replace('/', '|'): v for k, v in d.items()})\n")
    subprocess.check_call(["/opt/conda/bin/python3.9", "-c", code, src, dst])


if __name__ == "__main__":
    if len(sys.argv) > 1:            # e.g. gen_golden.py gen_ale_env
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    gen_phi()
    gen_phi_crop()
    gen_ale_env()
    gen_dqn_phi()
    gen_rmsprop()
    gen_checkpoint()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
