"""Test-side helpers: synthetic env pools and the oracle's view of the
lockstep windows the GPU runs on them (test infrastructure, uses oracle/)."""
import numpy as np

import oracle as O


def make_pools(rng, pool_len, n, kind="uniform", p_done=0.15):
    """pairs (pool_len, n, 2, 210, 160, 3) uint8 (frame 4, frame 3 of the
    skip); rewards (pool_len, n) f32 incl. out-of-range values (clip test);
    dones (pool_len, n) uint8.  kind: "uniform" [0, 255]; "palette" sparse
    palette blocks on black (SURVEY 8(d) variant ii, Breakout- / Space
    Invaders-shaped); "shaped": palette frames with every 16th env all-255
    (variant iii, luminance 254) and every 16th env (offset 9) uniform."""
    if kind == "uniform":
        pairs = rng.integers(0, 256, (pool_len, n, 2, 210, 160, 3), dtype=np.uint8)
    elif kind == "shaped":
        pairs, _, _ = make_pools(rng, pool_len, n, "palette", p_done)
        pairs[:, 5::16] = 255
        pairs[:, 9::16] = rng.integers(0, 256, pairs[:, 9::16].shape, dtype=np.uint8)
    else:
        pairs = np.zeros((pool_len, n, 2, 210, 160, 3), np.uint8)
        pal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
        for k in range(pool_len):
            for e in range(n):
                for f in range(2):
                    for _ in range(30):
                        y, x = rng.integers(0, 200), rng.integers(0, 150)
                        pairs[k, e, f, y:y + 8, x:x + 10] = pal[rng.integers(0, 16)]
    rewards = rng.choice(np.array([-2.0, -1.0, 0.0, 0.0, 0.0, 1.0, 3.5], np.float32), (pool_len, n))
    dones = (rng.random((pool_len, n)) < p_done).astype(np.uint8)
    return pairs, rewards.astype(np.float32), dones


class OracleEnvView:
    """Frame stacks the GPU's ring holds after observing pool steps 0..k
    (k = 0 force-reset; afterwards reset = done that came with the obs)."""

    def __init__(self, pairs, dones, mode=O.RESIZE_SCALAR):
        self.pairs, self.dones, self.mode = pairs, dones, mode
        self.pool_len, self.n = pairs.shape[0], pairs.shape[1]
        self.stacks = {}
        self._stack = None
        self._k = -1

    def stack(self, k):
        while self._k < k:
            self._k += 1
            j = self._k % self.pool_len
            scr = np.stack([O.current_screen(self.pairs[j, e, 0], self.pairs[j, e, 1], self.mode)
                            for e in range(self.n)])
            out = np.zeros((self.n, 4, 84, 84), np.uint8)
            for e in range(self.n):
                reset = self._k == 0 or self.dones[j, e] != 0
                out[e] = O.stack_push(None if reset else self._stack[e], scr[e], reset)
            self._stack = out
            self.stacks[self._k] = out
        return self.stacks[k]

    def states_f32(self, k0, T):
        return np.stack([O.PHI_LUT[self.stack(k0 + t)] for t in range(T)]), O.PHI_LUT[self.stack(k0 + T)]

    def window_rd(self, rewards, k0, T):
        idx = [(k0 + t + 1) % self.pool_len for t in range(T)]
        return rewards[idx].copy(), self.dones[idx].copy()


def make_rgb_pools(rng, pool_len, n, H=120, W=160, p_done=0.15):
    """ViZDoom-style pools: screens (pool_len, n, H, W, 3) uint8 RGB24
    (doom_env.py:47); rewards and dones as make_pools."""
    imgs = rng.integers(0, 256, (pool_len, n, H, W, 3), dtype=np.uint8)
    rewards = rng.choice(np.array([-2.0, -1.0, 0.0, 0.0, 0.0, 1.0, 3.5], np.float32), (pool_len, n))
    dones = (rng.random((pool_len, n)) < p_done).astype(np.uint8)
    return imgs, rewards.astype(np.float32), dones


class OracleRgbView(OracleEnvView):
    """States of an RGB net: phi of the current screen only
    (train_a3c_doom.py:21-23), no frame stack."""

    def __init__(self, imgs, dones, mode=O.RESIZE_SCALAR):
        self.imgs, self.dones, self.mode = imgs, dones, mode
        self.pool_len, self.n = imgs.shape[0], imgs.shape[1]

    def state(self, k):
        j = k % self.pool_len
        return np.stack([O.rgb_phi(self.imgs[j, e], self.mode) for e in range(self.n)])

    def states_f32(self, k0, T):
        return np.stack([self.state(k0 + t) for t in range(T)]), self.state(k0 + T)


def make_state_pools(rng, pool_len, n, p_done=0.15):
    """ARCH_STATES pools: float32 (pool_len, n, 4, 84, 84) states as a user
    phi might return them (signed, not an image of uint8 screens); rewards
    and dones as make_pools."""
    states = rng.standard_normal((pool_len, n, 4, 84, 84)).astype(np.float32)
    rewards = rng.choice(np.array([-2.0, -1.0, 0.0, 0.0, 0.0, 1.0, 3.5], np.float32), (pool_len, n))
    dones = (rng.random((pool_len, n)) < p_done).astype(np.uint8)
    return states, rewards.astype(np.float32), dones


class OracleStatesView(OracleEnvView):
    """States of an ARCH_STATES net: the pool entry itself (no phi, no stack)."""

    def __init__(self, states, dones):
        self.states, self.dones = states, dones
        self.pool_len, self.n = states.shape[0], states.shape[1]

    def states_f32(self, k0, T):
        P = self.pool_len
        return np.stack([self.states[(k0 + t) % P] for t in range(T)]), self.states[(k0 + T) % P]


def _sum_into(acc, g):
    for k, v in g.items():
        acc[k] = acc.get(k, 0.0) + v.astype(np.float64)


def oracle_window_chunks(arch, params, states, acts, r, d, boot, st=None, dprev=None, acts_dev=None, return_f64=False):
    """O.ff_window_grads / O.lstm_window over env chunks of 128 (envs are
    independent until the learner sums their gradients); gradients summed in
    f64 (returned as f32; return_f64=True keeps f64), per-env outputs
    concatenated, grad_mag = each element's summand norms in quadrature."""
    T, N = acts.shape
    CHUNK = 128
    g, aux, mag = {}, {}, {}
    for e0 in range(0, N, CHUNK):
        sl = slice(e0, min(N, e0 + CHUNK))
        da = tuple(a[:, sl].reshape((-1,) + a.shape[2:]) for a in acts_dev)
        if arch == O.ARCH_LSTM:
            s0 = O.LSTMState(h=st.h[sl], c=st.c[sl], has=st.has[sl])
            gc, ac = O.lstm_window(params, states[:, sl], acts[:, sl], r[:, sl], dprev[:, sl], d[:, sl], boot[sl], s0,
                                   dev_acts=da)
        else:
            gc, ac = O.ff_window_grads(params, states[:, sl], acts[:, sl], r[:, sl], d[:, sl], boot[sl],
                                       dev_acts=da)
        _sum_into(g, gc)
        for k, m in ac["grad_mag"].items():
            mag[k] = mag.get(k, 0.0) + m.astype(np.float64) ** 2
        for k in ("logits", "v", "dlogits", "dv"):
            aux.setdefault(k, []).append(ac[k])
        aux.setdefault("vboot", []).append(ac["vboot"])
        if arch == O.ARCH_LSTM:
            for k in ("h_last", "c_last"):
                aux.setdefault(k, []).append(ac[k])
    out = {k: np.concatenate(v, axis=0 if k in ("vboot", "h_last", "c_last") else 1) for k, v in aux.items()}
    out["grad_mag"] = {k: np.sqrt(v) for k, v in mag.items()}
    return ({k: v.astype(np.float64 if return_f64 else np.float32) for k, v in g.items()}), out
