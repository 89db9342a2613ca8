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


# --------------------------------------------------------------------------
# A3C update trajectories: a3c.py / policy_output.py / policy.py /
# v_function.py / dqn_head.py / init_like_torch.py / rmsprop_async.py and the
# model classes of a3c_ale.py:28-70 run verbatim on a torch-float64 Chainer
# stub (tests/golden/chainer_stub.py), driven like a3c_ale.py:100-126 over the
# reference's ALE wrapper on the scripted fake emulator.
# --------------------------------------------------------------------------
A3C_VARIANTS = {
    # name: (arch, kwargs of a3c.A3C, GradientClipping threshold, beta, n act calls, phi)
    # phi: "dqn" = the reference's dqn_phi (a3c_ale.py:220), "norm" = tests/a3c_golden.norm_phi,
    # a user phi through the plugin point (a3c.py:34,50,73) that is not dqn_phi's image
    "ff": ("ff", dict(pi_loss_coef=1.0, v_loss_coef=0.5, keep_loss_scale_same=False), 40.0, 1e-2, 44, "dqn"),
    "ff_opts": ("ff", dict(pi_loss_coef=0.5, v_loss_coef=1.0, keep_loss_scale_same=True), 0.05, 5e-2, 44, "dqn"),
    "lstm": ("lstm", dict(pi_loss_coef=1.0, v_loss_coef=0.5, keep_loss_scale_same=False), 40.0, 1e-2, 44, "dqn"),
    "lstm_opts": ("lstm", dict(pi_loss_coef=0.5, v_loss_coef=0.5, keep_loss_scale_same=True), 0.05, 1e-2, 44, "dqn"),
    "ff_phi": ("ff", dict(pi_loss_coef=1.0, v_loss_coef=0.5, keep_loss_scale_same=False), 40.0, 1e-2, 44, "norm"),
    "lstm_phi": ("lstm", dict(pi_loss_coef=1.0, v_loss_coef=0.5, keep_loss_scale_same=False), 0.02, 1e-2, 44,
                 "norm"),
}
A3C_T, A3C_GAMMA, A3C_SEED, A3C_LR, A3C_STEPS = 5, 0.99, 1234, 7e-4, 10 ** 4
A3C_INIT_SEED = 21     # oracle.init_like_torch(arch, A, default_rng(A3C_INIT_SEED)) = theta0
SUBSET_MIN, SUBSET_K = 16384, 2048   # tensors larger than this are stored on a fixed index subset


def _ref_model_classes():
    """A3CFF / A3CLSTM, a3c_ale.py:28-70, executed from the reference's own
    source text (the module as a whole does not parse on Python >= 3.7:
    `import async`, a3c_ale.py:20)."""
    import chainer
    import dqn_head, policy, v_function, a3c  # noqa: E401  (reference modules)
    from init_like_torch import init_like_torch
    with open(os.path.join(REF, "a3c_ale.py")) as f:
        lines = f.read().splitlines()
    block = "\n".join(lines[27:70])
    assert block.startswith("class A3CFF(") and "self.lstm.c.unchain_backward()" in lines[69]
    ns = dict(chainer=chainer, L=chainer.links, F=chainer.functions, np=np, dqn_head=dqn_head, policy=policy,
              v_function=v_function, a3c=a3c, init_like_torch=init_like_torch)
    exec(compile("\n" * 27 + block, os.path.join(REF, "a3c_ale.py"), "exec"), ns)
    return ns["A3CFF"], ns["A3CLSTM"]


def _subset_index(name, numel):
    return np.sort(np.random.default_rng(sum(map(ord, name))).choice(numel, SUBSET_K, replace=False))


def gen_a3c():
    import logging
    import chainer_stub
    chainer_stub.install()
    install_cv2_stub()
    install_ale_stub()
    sys.path.insert(0, REF)
    for k in [k for k in sys.modules if k in ("ale", "a3c", "policy_output", "policy")]:
        del sys.modules[k]
    import ale, a3c, rmsprop_async, policy_output  # noqa: E401  (reference modules)
    from dqn_phi import dqn_phi
    import chainer
    A3CFF, A3CLSTM = _ref_model_classes()

    class Capture(logging.Handler):          # the reference's own process-0 debug log (a3c.py:94-163)
        def __init__(self):
            super().__init__(logging.DEBUG)
            self.recs = []

        def emit(self, rec):
            self.recs.append((rec.msg, rec.args))

    out = {}
    from a3c_golden import norm_phi                                  # tests/a3c_golden.py
    for vname, (arch, kw, clip, beta, K, phi_name) in A3C_VARIANTS.items():
        np.random.seed(17)
        env = ale.ALE("fake.rom", seed=3, max_start_nullops=4)       # reference ALE on the fake emulator
        n_actions = env.number_of_actions
        np.random.seed(5)                                            # init_like_torch draws (a3c_ale.py:36,53)
        model = (A3CFF if arch == "ff" else A3CLSTM)(n_actions)
        # theta0 is then replaced by the oracle's seeded draw of the same
        # distribution, so the tests regenerate it instead of storing 3-5 MB
        init = oracle.init_like_torch(oracle.ARCH_FF if arch == "ff" else oracle.ARCH_LSTM, n_actions,
                                      np.random.default_rng(A3C_INIT_SEED))
        for n, p in model.namedparams():
            assert p.data.shape == init[n.lstrip("/")].shape, n
            p.data[...] = init[n.lstrip("/")]
        opt = rmsprop_async.RMSpropAsync(lr=A3C_LR, eps=1e-1, alpha=0.99)
        opt.setup(model)
        opt.add_hook(chainer.optimizer.GradientClipping(clip))
        phi = dqn_phi if phi_name == "dqn" else norm_phi
        agent = a3c.A3C(model, opt, A3C_T, A3C_GAMMA, beta=beta, process_idx=0, phi=phi, **kw)
        names = [n.lstrip("/") for n, _ in model.namedparams()]
        theta0 = {n.lstrip("/"): p.data.copy() for n, p in model.namedparams()}

        # sampling: np.random.multinomial (policy_output.py:27) draws from the
        # SAME Philox uniform the HIP sampler uses -- (seed; env 0, counter =
        # t_max * updates so far + step in window) -- by inverse CDF over the
        # f32 probabilities; the reference's epsneg shift is undone first
        n_upd = [0]

        def multinomial(n, pvals, size=None):
            ctr = A3C_T * n_upd[0] + (agent.t - agent.t_start)
            u = oracle.sample_uniforms(A3C_SEED, np.array([0]), ctr)
            p = (np.asarray(pvals, np.float64) + np.finfo(np.float32).epsneg).astype(np.float32)
            k = int(oracle.sample_from_uniform(p[None, :], u)[0])
            h = np.zeros(len(pvals), np.int64)
            h[k] = 1
            return h

        upd = []
        real_update = opt.update

        def update():
            g = {n.lstrip("/"): p.grad.copy() for n, p in agent.shared_model.namedparams()}
            real_update()
            n_upd[0] += 1
            upd.append((g, {n.lstrip("/"): p.data.copy() for n, p in agent.shared_model.namedparams()}))

        opt.update = update
        cap = Capture()
        lg = logging.getLogger("a3c")
        lg.setLevel(logging.DEBUG)
        lg.addHandler(cap)
        orig_mn = np.random.multinomial
        np.random.multinomial = multinomial
        states, rewards, terms, lrs, actions, calls_upd = [], [], [], [], [], []
        try:
            for k in range(K):                                       # a3c_ale.py:100-126
                global_t = k + 1
                lr = (A3C_STEPS - global_t - 1) / A3C_STEPS * A3C_LR
                agent.optimizer.lr = lr
                st = np.stack(env.state)
                states.append(st)
                rewards.append(float(env.reward))
                terms.append(bool(env.is_terminal))
                lrs.append(lr)
                nu = len(upd)
                a = agent.act(env.state, env.reward, env.is_terminal)
                calls_upd.append(len(upd) > nu)
                actions.append(-1 if a is None else int(a))
                if env.is_terminal:
                    env.initialize()
                else:
                    env.receive_action(a)
        finally:
            np.random.multinomial = orig_mn
            lg.removeHandler(cap)
        # per-call policy outputs from the debug lines 't:%s entropy:%s, probs:%s' (a3c.py:161-163)
        probs = np.full((K, n_actions), np.nan)
        ent = np.full(K, np.nan)
        ci = [k for k in range(K) if actions[k] >= 0]
        steplog = [r for r in cap.recs if r[0].startswith("t:")]
        assert len(steplog) == len(ci)
        for k, (_, args) in zip(ci, steplog):
            ent[k] = float(np.asarray(args[1]).ravel()[0])
            probs[k] = np.asarray(args[2]).ravel()
        # per-update records: R per step ('s:%s v:%s R:%s'), losses, grad norm
        Rs, vs, losses, norms = [], [], [], []
        cur_R, cur_v = [], []
        for msg, args in cap.recs:
            if msg.startswith("s:"):
                cur_v.append(float(np.asarray(args[1]).ravel()[0]))
                cur_R.append(float(args[2]))
            elif msg.startswith("pi_loss"):
                losses.append((float(np.asarray(args[0]).ravel()[0]), float(np.asarray(args[1]).ravel()[0])))
                Rs.append(cur_R[::-1])
                vs.append(cur_v[::-1])
                cur_R, cur_v = [], []
            elif msg.startswith("grad norm"):
                norms.append(float(args[0]))
        U = len(upd)
        assert U == len(Rs) == len(norms) and U >= 6, (U, len(Rs), len(norms))
        pref = vname + "|"
        out[pref + "arch"] = np.array(arch)
        out[pref + "phi"] = np.array(phi_name)
        out[pref + "names"] = np.array(names)
        out[pref + "kw"] = np.array([kw["pi_loss_coef"], kw["v_loss_coef"], float(kw["keep_loss_scale_same"]),
                                     clip, beta, A3C_GAMMA, A3C_T, A3C_SEED, n_actions, A3C_INIT_SEED])
        st = np.stack(states)
        skey = "states|" + arch      # the fake emulator's frames ignore the actions: one copy per arch
        if skey in out:
            assert np.array_equal(out[skey], st)
        out[skey] = st
        out[pref + "rewards"] = np.array(rewards, np.float32)
        out[pref + "terminals"] = np.array(terms)
        out[pref + "lr"] = np.array(lrs)
        out[pref + "actions"] = np.array(actions, np.int32)
        out[pref + "probs"] = probs
        out[pref + "entropy"] = ent
        out[pref + "updates"] = np.array([k for k in range(K) if calls_upd[k]], np.int32)
        Rm = np.full((U, A3C_T), np.nan)
        vm = np.full((U, A3C_T), np.nan)
        for u in range(U):
            Rm[u, :len(Rs[u])] = Rs[u]
            vm[u, :len(vs[u])] = vs[u]
        out[pref + "R"] = Rm
        out[pref + "v"] = vm
        out[pref + "loss"] = np.array(losses)
        out[pref + "grad_norm"] = np.array(norms)
        for n in names:
            g = np.stack([u[0][n] for u in upd])
            p = np.stack([u[1][n] for u in upd])
            if theta0[n].size > SUBSET_MIN:
                idx = _subset_index(n, theta0[n].size)
                out[pref + "idx|" + n] = idx
                g = g.reshape(U, -1)[:, idx]
                p = p.reshape(U, -1)[:, idx]
            out[pref + "grad|" + n] = g
            out[pref + "param|" + n] = p
        print(vname, "calls", K, "updates", U, "terminal updates",
              int(sum(terms[k] for k in range(K) if calls_upd[k])), "norms", np.round(norms, 3))
    np.savez_compressed(os.path.join(HERE, "a3c_update_golden.npz"), **out)
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
