"""Shared access to tests/golden/a3c_update_golden.npz: A3C.act trajectories
of the REFERENCE's own a3c.py / policy_output.py / policy.py / v_function.py /
dqn_head.py / rmsprop_async.py and a3c_ale.py's model classes, run on a
torch-float64 Chainer stub by tests/golden/gen_golden.py (gen_a3c), driven
like a3c_ale.py:100-126 over the reference's ALE wrapper on a scripted fake
emulator.  Per variant: the act calls' inputs (ALE.state, reward, terminal,
lr), the returned actions, the policy outputs, and per update the returns,
values, losses, grad norm, gradients and post-update parameters (tensors
above 16,384 elements on a fixed index subset)."""
import os

import numpy as np

import oracle as O

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "a3c_update_golden.npz")
VARIANTS = ("ff", "ff_opts", "lstm", "lstm_opts", "ff_phi", "lstm_phi")


def norm_phi(screens):
    """The *_phi variants' phi (a3c.py:34,50,73 plugin point): the 4 uint8
    screens to float32 in [-1, 1] -- not dqn_phi's image of them.  The
    generator hands this very function to the reference's a3c.A3C."""
    x = np.asarray(screens, dtype=np.float32)
    x /= np.float32(127.5)
    x -= np.float32(1.0)
    return x


class Variant:
    def __init__(self, z, name):
        pre = name + "|"
        self.name = name
        self.arch_name = str(z[pre + "arch"])
        self.phi_name = str(z[pre + "phi"]) if pre + "phi" in z.files else "dqn"
        self.phi = None if self.phi_name == "dqn" else norm_phi
        self.arch = O.ARCH_FF if self.arch_name == "ff" else O.ARCH_LSTM
        (self.pi_loss_coef, self.v_loss_coef, keep, self.clip, self.beta, self.gamma, T, seed, A,
         init_seed) = z[pre + "kw"]
        self.keep = bool(keep)
        self.T, self.seed, self.A, self.init_seed = int(T), int(seed), int(A), int(init_seed)
        self.names = [str(n) for n in z[pre + "names"]]
        self.states = z["states|" + self.arch_name]
        self.rewards = z[pre + "rewards"]
        self.terminals = z[pre + "terminals"]
        self.lr = z[pre + "lr"]
        self.actions = z[pre + "actions"]
        self.probs = z[pre + "probs"]
        self.entropy = z[pre + "entropy"]
        self.update_calls = z[pre + "updates"]
        self.R, self.v = z[pre + "R"], z[pre + "v"]
        self.loss, self.grad_norm = z[pre + "loss"], z[pre + "grad_norm"]
        self.grad = {n: z[pre + "grad|" + n] for n in self.names}
        self.param = {n: z[pre + "param|" + n] for n in self.names}
        self.idx = {n: z[pre + "idx|" + n] for n in self.names if pre + "idx|" + n in z.files}

    @property
    def n_calls(self):
        return len(self.actions)

    def theta0(self):
        return O.init_like_torch(self.arch, self.A, np.random.default_rng(self.init_seed))

    def pick(self, name, full):
        """The stored elements of one tensor (its index subset if it has one)."""
        a = np.asarray(full).reshape(-1)
        return a[self.idx[name]] if name in self.idx else np.asarray(full).reshape(self.grad[name].shape[1:])

    def window_lengths(self):
        out, t, t_start = [], 0, 0
        for k in range(self.n_calls):
            if k in set(self.update_calls.tolist()):
                out.append(t - t_start)
                t_start = t
            if self.actions[k] >= 0:
                t += 1
        return out


def load(name):
    with np.load(PATH) as z:
        return Variant(z, name)
