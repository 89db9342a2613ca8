"""CPU oracle: a NumPy restatement of the reference A3C hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (`async-rl_amd/`)
imports this module.  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may use it, and only as the checker / the
timed CPU baseline -- never as the thing measured or shipped.

Every function restates one piece of PeerM/async-rl (reference @ v0) and cites
the file:line it follows.  Where the arithmetic lives in a third-party library
that is absent here (Chainer 1.8.1, pinned in README.md:53; OpenCV, unpinned),
the function restates that library's published algorithm and says so.

Pinning (see DESIGN.md "Oracle"):
  * luminance / max-pool / frame stack / dqn_phi: pinned bit-exact by golden
    vectors produced by the reference's own code (tests/golden/gen_golden.py
    imports /root/reference/dqn_phi.py directly and runs ale.py's
    current_screen with stub ALE/cv2 modules).
  * RMSpropAsync.update_one_cpu: pinned by golden vectors from the reference's
    own rmsprop_async.py run on NumPy arrays through a minimal chainer stub.
  * OpenCV INTER_LINEAR resize: parity UNPINNED (OpenCV absent, version
    unpinned); the scalar FixedPtCast path is declared canonical.
  * Chainer conv/linear/LSTM/softmax/autograd: parity UNPINNED by reference
    fixtures (Chainer absent); restated from Chainer 1.8.1 semantics and
    cross-checked against torch-CPU autograd in tests/test_oracle.py.  The
    trained Breakout checkpoint (tests/golden/breakout_ff.npz) supplies real
    weights.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

F32 = np.float32

# ----------------------------------------------------------------------------
# Phi: ale.py:59-89, ale.py:111-161, dqn_phi.py:4-17
# ----------------------------------------------------------------------------

SRC_H, SRC_W = 210, 160
DST = 84


def max_pool_pair(cur: np.ndarray, prev: np.ndarray) -> np.ndarray:
    """ale.py:62 -- np.maximum of the two captured RGB frames (uint8)."""
    return np.maximum(cur, prev)


def luminance_u8(rgb: np.ndarray) -> np.ndarray:
    """ale.py:67-69 -- float64 R*0.2126 + G*0.0722 + B*0.7152 (left to
    right), then astype(uint8) truncation.  Note G/B weights are swapped
    relative to Rec.709; reproduced as written."""
    r = rgb[..., 0] * 0.2126
    g = rgb[..., 1] * 0.0722
    b = rgb[..., 2] * 0.7152
    return ((r + g) + b).astype(np.uint8)


def resize_coeffs(ssize: int, dsize: int):
    """OpenCV (unpinned; restated from the 3.x/4.x generic resize path)
    INTER_LINEAR fixed-point coefficients for one axis, as called from
    ale.py:84-85 (cv2.resize(img, (84, 84), INTER_LINEAR)).

    scale = 1/(dsize/ssize) in double; f = (float)((d+0.5)*scale-0.5);
    s = floor(f); f -= s; clamp at borders; alpha = saturate_cast<short>
    ((1-f)*2048), (f*2048) with round-half-even (cvRound)."""
    inv_scale = float(dsize) / float(ssize)
    scale = 1.0 / inv_scale
    ofs = np.zeros(dsize, np.int32)
    alpha = np.zeros((dsize, 2), np.int32)
    for d in range(dsize):
        f = F32((d + 0.5) * scale - 0.5)
        s = int(math.floor(float(f)))
        f = F32(f - F32(s))
        if s < 0:
            f, s = F32(0.0), 0
        if s >= ssize - 1:
            f, s = F32(0.0), ssize - 1
        c0 = F32(F32(1.0) - f)
        c1 = f
        a0 = int(np.rint(F32(c0 * F32(2048.0))))
        a1 = int(np.rint(F32(c1 * F32(2048.0))))
        ofs[d] = s
        alpha[d] = (a0, a1)
    return ofs, alpha


_XOFS, _XALPHA = resize_coeffs(SRC_W, DST)
_YOFS, _YBETA = resize_coeffs(SRC_H, DST)

RESIZE_SCALAR = 0   # FixedPtCast<int,uchar,22>: (b0*r0 + b1*r1 + 2^21) >> 22
RESIZE_SIMD = 1     # VResizeLinearVec_32s8u: ((r0>>4)*b0>>16)+((r1>>4)*b1>>16)+2 >> 2
RESIZE_CROP = 2     # flag: ale.py:73-82 -- cv2.resize(img, (84, 110)), keep rows [18, 102)

_CROP_TOP = (110 - 84) - 8                       # ale.py:78-80: unused_height - bottom_crop
_YOFS_C, _YBETA_C = (a[_CROP_TOP:_CROP_TOP + DST] for a in resize_coeffs(SRC_H, 110))


def resize_linear_u8(img: np.ndarray, mode: int = RESIZE_SCALAR) -> np.ndarray:
    """cv2.resize(img, (84,84), INTER_LINEAR) for a (..., 210, 160) uint8
    plane (ale.py:84-85).  Horizontal pass: int row = S[sx]*a0 + S[sx+1]*a1
    (HResizeLinear, exact); vertical pass per `mode` (bit 0: SIMD form).
    mode & RESIZE_CROP: rows 18..101 of cv2.resize(img, (84, 110)) instead
    (ale.py:73-82) -- the same passes with the 210 -> 110 row coefficients."""
    src = img.astype(np.int64)
    xs = _XOFS
    xs1 = np.minimum(xs + 1, SRC_W - 1)
    rows = src[..., :, xs] * _XALPHA[:, 0] + src[..., :, xs1] * _XALPHA[:, 1]
    yofs, ybeta = (_YOFS_C, _YBETA_C) if mode & RESIZE_CROP else (_YOFS, _YBETA)
    ys = yofs
    ys1 = np.minimum(ys + 1, SRC_H - 1)
    r0 = rows[..., ys, :]
    r1 = rows[..., ys1, :]
    b0 = ybeta[:, 0][:, None]
    b1 = ybeta[:, 1][:, None]
    mode &= ~RESIZE_CROP
    if mode == RESIZE_SCALAR:
        out = (b0 * r0 + b1 * r1 + (1 << 21)) >> 22
    elif mode == RESIZE_SIMD:
        out = ((((r0 >> 4) * b0) >> 16) + (((r1 >> 4) * b1) >> 16) + 2) >> 2
    else:
        raise ValueError("resize mode must be 0 (scalar) or 1 (simd)")
    return np.clip(out, 0, 255).astype(np.uint8)


def resize_linear_any_u8(img: np.ndarray, mode: int = RESIZE_SCALAR) -> np.ndarray:
    """cv2.resize(img, (84, 84), INTER_LINEAR) of a (..., H, W) uint8 plane of
    any size: the same two fixed-point passes as resize_linear_u8 with the
    coefficients of H -> 84 and W -> 84 (OpenCV resizes each channel of an
    8UC3 image with one coefficient set: HResizeLinear indexes sx*cn + k)."""
    H, W = img.shape[-2:]
    xs, xa = resize_coeffs(W, DST)
    ys, yb = resize_coeffs(H, DST)
    src = img.astype(np.int64)
    rows = src[..., :, xs] * xa[:, 0] + src[..., :, np.minimum(xs + 1, W - 1)] * xa[:, 1]
    r0 = rows[..., ys, :]
    r1 = rows[..., np.minimum(ys + 1, H - 1), :]
    b0 = yb[:, 0][:, None]
    b1 = yb[:, 1][:, None]
    if mode == RESIZE_SCALAR:
        out = (b0 * r0 + b1 * r1 + (1 << 21)) >> 22
    elif mode == RESIZE_SIMD:
        out = ((((r0 >> 4) * b0) >> 16) + (((r1 >> 4) * b1) >> 16) + 2) >> 2
    else:
        raise ValueError("resize mode must be 0 (scalar) or 1 (simd)")
    return np.clip(out, 0, 255).astype(np.uint8)


def rgb_screen_u8(img: np.ndarray, mode: int = RESIZE_SCALAR) -> np.ndarray:
    """train_a3c_doom.py:22-23 up to the uint8 planes: cv2.resize of the
    (H, W, 3) RGB24 screen (doom_env.py:47) to (84, 84, 3), transposed to
    (3, 84, 84)."""
    assert img.ndim == 3 and img.shape[2] == 3
    return resize_linear_any_u8(np.moveaxis(img, 2, 0), mode)


def rgb_phi(img: np.ndarray, mode: int = RESIZE_SCALAR) -> np.ndarray:
    """train_a3c_doom.py:21-23: phi(obs) = resize -> transpose(2, 0, 1) ->
    astype(float32) / 255 (f32 true division)."""
    return rgb_screen_u8(img, mode).astype(np.float32) / F32(255.0)


def current_screen(cur: np.ndarray, prev: np.ndarray,
                   mode: int = RESIZE_SCALAR) -> np.ndarray:
    """ale.py:59-89 (crop_or_scale='scale', the default at ale.py:18; 'crop'
    with mode | RESIZE_CROP): max of two frames -> luminance -> uint8 ->
    84x84 resize."""
    assert cur.shape[-3:] == (SRC_H, SRC_W, 3)
    return resize_linear_u8(luminance_u8(max_pool_pair(cur, prev)), mode)


def stack_push(stack: np.ndarray, plane: np.ndarray, reset: bool) -> np.ndarray:
    """ale.py:155-158 (reset: three zero planes + the new screen) and
    ale.py:135 (deque(maxlen=4).append).  Oldest plane first."""
    if reset:
        out = np.zeros((4, DST, DST), np.uint8)
        out[3] = plane
        return out
    return np.concatenate([stack[1:], plane[None]], axis=0)


def dqn_phi(screens) -> np.ndarray:
    """dqn_phi.py:4-17: asarray(float32) then in-place /= 255.0 (IEEE f32)."""
    assert len(screens) == 4
    raw = np.asarray(screens, dtype=np.float32)
    raw /= F32(255.0)
    return raw


PHI_LUT = (np.arange(256, dtype=np.float32) / F32(255.0)).astype(np.float32)

# ----------------------------------------------------------------------------
# Model parameters: a3c_ale.py:28-70, dqn_head.py:31-52, policy.py:32-58,
# v_function.py:10-34, init_like_torch.py:5-22
# ----------------------------------------------------------------------------

ARCH_FF = 0
ARCH_LSTM = 1
ARCH_FF_NATURE = 2     # A3CFF with NatureDQNHead (dqn_head.py:6-28) instead of NIPSDQNHead
ARCH_RGB = 16          # flag (FF / LSTM): the ViZDoom models, train_a3c_doom.py:25-63 --
                       # NIPSDQNHead(n_input_channels=3) on one RGB screen


def param_shapes(arch: int, n_actions: int):
    """Chainer namedparams / HDF5 paths in link order (a3c_ale.py:35,52;
    train_a3c_doom.py:28-33,46-53 for the RGB models)."""
    c_in = 3 if arch & ARCH_RGB else 4
    arch &= ~ARCH_RGB
    head = [("0/0/W", (16, c_in, 8, 8)), ("0/0/b", (16,)),
            ("0/1/W", (32, 16, 4, 4)), ("0/1/b", (32,)),
            ("0/2/W", (256, 2592)), ("0/2/b", (256,))]
    if arch == ARCH_FF:
        return head + [("1/0/W", (n_actions, 256)), ("1/0/b", (n_actions,)),
                       ("2/0/W", (1, 256)), ("2/0/b", (1,))]
    if arch == ARCH_FF_NATURE:   # dqn_head.py:16-20 (4->32 k8s4, 32->64 k4s2, 64->64 k3s1, 3136->512)
        return [("0/0/W", (32, 4, 8, 8)), ("0/0/b", (32,)), ("0/1/W", (64, 32, 4, 4)), ("0/1/b", (64,)),
                ("0/2/W", (64, 64, 3, 3)), ("0/2/b", (64,)), ("0/3/W", (512, 3136)), ("0/3/b", (512,)),
                ("1/0/W", (n_actions, 512)), ("1/0/b", (n_actions,)), ("2/0/W", (1, 512)), ("2/0/b", (1,))]
    if arch == ARCH_LSTM:
        return head + [("1/upward/W", (1024, 256)), ("1/upward/b", (1024,)),
                       ("1/lateral/W", (1024, 256)),
                       ("2/0/W", (n_actions, 256)), ("2/0/b", (n_actions,)),
                       ("3/0/W", (1, 256)), ("3/0/b", (1,))]
    raise ValueError(arch)


def pname(arch: int, role: str) -> str:
    """Short role names -> namedparam paths."""
    arch &= ~ARCH_RGB
    if arch == ARCH_FF:
        m = {"c1W": "0/0/W", "c1b": "0/0/b", "c2W": "0/1/W", "c2b": "0/1/b",
             "fcW": "0/2/W", "fcb": "0/2/b", "piW": "1/0/W", "pib": "1/0/b",
             "vW": "2/0/W", "vb": "2/0/b"}
    elif arch == ARCH_FF_NATURE:
        m = {"c1W": "0/0/W", "c1b": "0/0/b", "c2W": "0/1/W", "c2b": "0/1/b",
             "c3W": "0/2/W", "c3b": "0/2/b", "fcW": "0/3/W", "fcb": "0/3/b",
             "piW": "1/0/W", "pib": "1/0/b", "vW": "2/0/W", "vb": "2/0/b"}
    else:
        m = {"c1W": "0/0/W", "c1b": "0/0/b", "c2W": "0/1/W", "c2b": "0/1/b",
             "fcW": "0/2/W", "fcb": "0/2/b", "luW": "1/upward/W",
             "lub": "1/upward/b", "llW": "1/lateral/W", "piW": "2/0/W",
             "pib": "2/0/b", "vW": "3/0/W", "vb": "3/0/b"}
    return m[role]


def init_like_torch(arch: int, n_actions: int, rng: np.random.Generator):
    """init_like_torch.py:5-22: U(-1/sqrt(fan_in), +1/sqrt(fan_in)) for W and
    b of every Linear / Convolution2D; fan_in = in*kh*kw.  (Same distribution,
    a seeded Generator instead of the global RNG.)"""
    params = {}
    shapes = dict(param_shapes(arch, n_actions))
    for name, shape in param_shapes(arch, n_actions):
        wshape = shapes[name.rsplit("/", 1)[0] + "/W"]
        fan_in = int(np.prod(wshape[1:]))
        stdv = 1.0 / np.sqrt(fan_in)
        params[name] = rng.uniform(-stdv, stdv, size=shape).astype(np.float32)
    return params


# ----------------------------------------------------------------------------
# Forward (Chainer 1.8.1 semantics, restated)
# ----------------------------------------------------------------------------

def _im2col(x: np.ndarray, k: int, s: int):
    """Chainer conv.im2col_cpu layout: (N, C, kh, kw, OH, OW) -> we return
    (N, OH, OW, C*kh*kw) rows (cross-correlation, no padding)."""
    n, c, h, w = x.shape
    oh = (h - k) // s + 1
    ow = (w - k) // s + 1
    st = x.strides
    view = np.lib.stride_tricks.as_strided(
        x, shape=(n, oh, ow, c, k, k),
        strides=(st[0], st[2] * s, st[3] * s, st[1], st[2], st[3]),
        writeable=False)
    return np.ascontiguousarray(view).reshape(n, oh, ow, c * k * k), oh, ow


def conv2d(x: np.ndarray, W: np.ndarray, b: np.ndarray, s: int) -> np.ndarray:
    """L.Convolution2D forward (dqn_head.py:41-42): tensordot(col, W) + b."""
    oc, ic, k, _ = W.shape
    cols, oh, ow = _im2col(x, k, s)
    y = cols.reshape(-1, ic * k * k) @ W.reshape(oc, -1).T
    y = y.astype(np.float32) + b
    return y.reshape(x.shape[0], oh, ow, oc).transpose(0, 3, 1, 2).copy()


def conv2d_backward(x, W, gy, s, need_dx=True, mag=None, names=None):
    """Gradient of conv2d w.r.t. W, b and (optionally) x.  mag (dict) +
    names (W, b): also store the L2 norm of each gradient element's summands
    (grad_mag)."""
    oc, ic, k, _ = W.shape
    n = x.shape[0]
    cols, oh, ow = _im2col(x, k, s)
    gyf = gy.transpose(0, 2, 3, 1).reshape(-1, oc)
    gW = gmm(gyf.T, cols.reshape(-1, ic * k * k)).reshape(W.shape)
    gb = gsum(gyf)
    if mag is not None:
        mag[names[0]] = _mag_mm(gyf.T, cols.reshape(-1, ic * k * k)).reshape(W.shape)
        mag[names[1]] = _mag_sum(gyf)
    gx = None
    if need_dx:
        gcol = (gyf @ W.reshape(oc, -1)).reshape(n, oh, ow, ic, k, k)
        gx = np.zeros_like(x)
        for ky in range(k):
            for kx in range(k):
                gx[:, :, ky:ky + s * oh:s, kx:kx + s * ow:s] += \
                    gcol[:, :, :, :, ky, kx].transpose(0, 3, 1, 2)
    return gW.astype(np.float32), gb.astype(np.float32), gx


def relu(x):
    return np.maximum(x, F32(0.0))


# Weight-gradient reductions (sums over samples and positions, up to millions
# of terms at the bench configs) are accumulated in float64 and rounded to
# f32 once, so the oracle's own summation error stays far below the HIP
# path's; the summands themselves are the f32 values of the restated graph.
# The CPU baseline (oracle/cpu_baseline.py) sets this False to time
# Chainer's f32 arithmetic.
EXACT_SUMS = True


def gmm(a, b):
    """a @ b for a gradient reduction (float64 accumulation when EXACT_SUMS)."""
    if EXACT_SUMS:
        return (np.asarray(a, np.float64) @ np.asarray(b, np.float64)).astype(np.float32)
    return (a @ b).astype(np.float32)


def gsum(a, axis=0):
    """Sum for a bias gradient (float64 accumulation when EXACT_SUMS)."""
    return np.asarray(a).sum(axis=axis, dtype=np.float64 if EXACT_SUMS else np.float32).astype(np.float32)


def linear(x, W, b=None):
    """L.Linear: y = x.dot(W.T) (+ b)."""
    y = (x @ W.T).astype(np.float32)
    if b is not None:
        y = y + b
    return y


def nips_head(params, arch, x):
    """NIPSDQNHead.__call__ (dqn_head.py:48-52): conv(8,s4) -> relu ->
    conv(4,s2) -> relu -> Linear(2592,256) -> relu.  Returns activations."""
    a1 = relu(conv2d(x, params[pname(arch, "c1W")], params[pname(arch, "c1b")], 4))
    a2 = relu(conv2d(a1, params[pname(arch, "c2W")], params[pname(arch, "c2b")], 2))
    h = relu(linear(a2.reshape(a2.shape[0], -1), params[pname(arch, "fcW")],
                    params[pname(arch, "fcb")]))
    return a1, a2, h


def nature_head(params, x):
    """NatureDQNHead.__call__ (dqn_head.py:24-28): conv(4->32, 8, s4) -> relu
    -> conv(32->64, 4, s2) -> relu -> conv(64->64, 3, s1) -> relu ->
    Linear(3136, 512) -> relu.  Returns the activations (a1, a2, a3, h)."""
    arch = ARCH_FF_NATURE
    a1 = relu(conv2d(x, params[pname(arch, "c1W")], params[pname(arch, "c1b")], 4))
    a2 = relu(conv2d(a1, params[pname(arch, "c2W")], params[pname(arch, "c2b")], 2))
    a3 = relu(conv2d(a2, params[pname(arch, "c3W")], params[pname(arch, "c3b")], 1))
    h = relu(linear(a3.reshape(a3.shape[0], -1), params[pname(arch, "fcW")],
                    params[pname(arch, "fcb")]))
    return a1, a2, a3, h


def sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(np.float32)


def lstm_cell(params, arch, x, h_prev, c_prev, has_state):
    """Chainer 1.8.1 L.LSTM.__call__ + F.lstm (a3c_ale.py:50-51,59,62):
    lstm_in = upward(x) [+ lateral(h) if h is not None]; gates interleaved
    (reshape(N, 256, 4)): a,i,f,o = [:, :, 0..3]; c = tanh(a)*sig(i) +
    sig(f)*c_prev; h = sig(o)*tanh(c).  has_state (N,) bool: False = state
    is None (after reset_state, a3c_ale.py:65-66)."""
    g = linear(x, params[pname(arch, "luW")], params[pname(arch, "lub")])
    m = has_state.astype(np.float32)[:, None]
    g = g + linear(h_prev * m, params[pname(arch, "llW")])
    a = np.tanh(g[:, 0::4])
    i = sigmoid(g[:, 1::4])
    f = sigmoid(g[:, 2::4])
    o = sigmoid(g[:, 3::4])
    c = a * i + f * (c_prev * m)
    h = o * np.tanh(c)
    return g, c.astype(np.float32), h.astype(np.float32)


def softmax(z):
    """F.softmax (policy_output.py:41-43): max-subtracted exp, normalised."""
    y = z - z.max(axis=1, keepdims=True)
    y = np.exp(y)
    return (y / y.sum(axis=1, keepdims=True)).astype(np.float32)


def log_softmax(z):
    """F.log_softmax (policy_output.py:45-47): x - logsumexp(x)."""
    m = z.max(axis=1, keepdims=True)
    s = np.log(np.exp(z - m).sum(axis=1, keepdims=True))
    return (z - (m + s)).astype(np.float32)


def entropy(p, logp):
    """policy_output.py:59-61: -sum(p * log p)."""
    return (-(p * logp).sum(axis=-1)).astype(np.float32)


def pi_and_v_ff(params, x, arch=ARCH_FF):
    """A3CFF.pi_and_v (a3c_ale.py:38-40); arch=ARCH_FF_NATURE swaps in the
    Nature head (hidden 512)."""
    acts = nature_head(params, x) if arch == ARCH_FF_NATURE else nips_head(params, ARCH_FF, x)
    h = acts[-1]
    logits = linear(h, params["1/0/W"], params["1/0/b"])
    v = linear(h, params["2/0/W"], params["2/0/b"])[:, 0]
    return logits, v, acts


# ----------------------------------------------------------------------------
# Sampling: policy_output.py:12-29 (distributional parity); Philox4x32-10
# ----------------------------------------------------------------------------

_PM0, _PM1 = 0xD2511F53, 0xCD9E8D57
_PW0, _PW1 = 0x9E3779B9, 0xBB67AE85
_M32 = 0xFFFFFFFF


def philox4x32(ctr, key, rounds=10):
    """Philox4x32-10 (Salmon et al. 2011).  ctr: (4, n) uint64 arrays of
    32-bit words; key: (2,) ints.  Returns (4, n) uint64 of 32-bit words."""
    c0, c1, c2, c3 = [np.asarray(c, np.uint64) & _M32 for c in ctr]
    k0 = np.uint64(key[0] & _M32)
    k1 = np.uint64(key[1] & _M32)
    for r in range(rounds):
        p0 = c0 * np.uint64(_PM0)
        p1 = c2 * np.uint64(_PM1)
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(_M32)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(_M32)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        if r != rounds - 1:
            k0 = (k0 + np.uint64(_PW0)) & np.uint64(_M32)
            k1 = (k1 + np.uint64(_PW1)) & np.uint64(_M32)
    return c0, c1, c2, c3


def sample_uniforms(seed: int, env_ids: np.ndarray, step: int) -> np.ndarray:
    """One U[0,1) f32 per env: Philox(ctr=(env, step_lo, step_hi, 0),
    key=(seed_lo, seed_hi)), u = (word0 >> 8) * 2^-24."""
    env_ids = np.asarray(env_ids, np.uint64)
    n = env_ids.shape[0]
    ctr = (env_ids, np.full(n, step & _M32, np.uint64),
           np.full(n, (step >> 32) & _M32, np.uint64), np.zeros(n, np.uint64))
    w0, _, _, _ = philox4x32(ctr, (seed & _M32, (seed >> 32) & _M32))
    return ((w0 >> np.uint64(8)).astype(np.float32) * F32(2.0 ** -24)).astype(np.float32)


def sample_from_uniform(probs: np.ndarray, u: np.ndarray) -> np.ndarray:
    """Inverse-CDF draw: first k with u < cumsum_f32(p)[k] (sequential f32
    adds), else A-1.  Distributionally equal to np.random.multinomial(1, p)
    at policy_output.py:26-28 (which first subtracts epsneg, :24)."""
    n, a = probs.shape
    out = np.full(n, a - 1, np.int32)
    cdf = np.zeros(n, np.float32)
    done = np.zeros(n, bool)
    for k in range(a):
        cdf = (cdf + probs[:, k]).astype(np.float32)
        hit = (~done) & (u < cdf)
        out[hit] = k
        done |= hit
    return out


# ----------------------------------------------------------------------------
# n-step return, losses and their gradient: a3c.py:82-126
# ----------------------------------------------------------------------------

def segment_scale(dones, t_max, valid=None):
    """a3c.py:116-121 (keep_loss_scale_same): the losses of a window that a
    terminal closed after len < t_max steps are scaled by t_max / len.  In a
    lockstep window every segment closed by a terminal is such a window; the
    segment running into the window end is not scaled.  Returns (T, N) f64."""
    T, N = dones.shape
    valid = np.ones((T, N), bool) if valid is None else valid
    scale = np.ones((T, N), np.float64)
    for e in range(N):
        start = 0
        for t in range(T):
            if not valid[t, e]:
                break
            if dones[t, e]:
                ln = t - start + 1
                if ln < t_max:
                    scale[start:t + 1, e] = t_max / ln
                start = t + 1
    return scale


def returns_and_lossgrad(rewards, dones, values, vboot, probs, logp, actions,
                         gamma=0.99, beta=0.01, v_loss_coef=0.5,
                         clip_reward=True, pi_loss_coef=1.0,
                         keep_loss_scale_same=False, t_max=None, valid=None):
    """Batched restatement of a3c.py:82-126 over a lockstep window.

    rewards, dones: (T, N) -- reward / terminal of transition t -> t+1
    values: (T, N) f32 v(s_t); vboot: (N,) f32 v(s_T) (pre-update params)
    probs, logp: (T, N, A); actions: (T, N).
    R is accumulated in float64 like the Python float at a3c.py:83-92; each
    terminal restarts it at 0 (a segment per episode, a3c.py:82-83).
    pi_loss_coef / v_loss_coef scale the two losses (a3c.py:110-114);
    keep_loss_scale_same scales terminal-closed segments shorter than t_max
    (default T) by t_max / len (a3c.py:116-121); valid (T, N) bool marks the
    steps that belong to the window (the rest get no loss).
    Returns R (f32), advantage, dlogits (T,N,A), dv (T,N), pi_loss, v_loss.
    """
    T, N = rewards.shape
    A = probs.shape[2]
    t_max = T if t_max is None else t_max
    valid = np.ones((T, N), bool) if valid is None else np.asarray(valid, bool)
    r = np.asarray(rewards, np.float64)
    if clip_reward:
        r = np.clip(r, -1, 1)                     # a3c.py:69-70
    R = vboot.astype(np.float64).copy()
    Rs = np.zeros((T, N), np.float32)
    for t in reversed(range(T)):
        R = np.where(dones[t] != 0, 0.0, R)       # a3c.py:82-83 (R=0 at terminal)
        R = R * gamma + r[t]                      # a3c.py:91-92
        Rs[t] = R.astype(np.float32)
    adv = (Rs - values).astype(np.float32)        # a3c.py:97 (f32 AddConstant)
    H = entropy(probs, logp)
    onehot = np.zeros_like(probs)
    np.put_along_axis(onehot, actions[..., None].astype(np.int64), 1.0, axis=2)
    scale = segment_scale(dones, t_max, valid) if keep_loss_scale_same else np.ones((T, N))
    pf = (F32(pi_loss_coef) * scale.astype(np.float32)).astype(np.float32) * valid
    vf = (F32(v_loss_coef) * scale.astype(np.float32)).astype(np.float32) * valid
    # d/dz of [-logpi(a)*adv - beta*H]  (a3c.py:103,105)
    dlogits = (pf[..., None] * (-adv[..., None] * (onehot - probs)
               + F32(beta) * probs * (logp + H[..., None]))).astype(np.float32)
    dv = (vf * (values - Rs)).astype(np.float32)   # a3c.py:108,113-114
    logp_a = np.take_along_axis(logp, actions[..., None].astype(np.int64), 2)[..., 0]
    pi_loss = float(-(pf * (logp_a * adv + F32(beta) * H)).sum())
    v_loss = float((vf * (((values - Rs) ** 2) / 2)).sum())
    return Rs, adv, dlogits, dv, pi_loss, v_loss


# ----------------------------------------------------------------------------
# Backward (total_loss.backward(), a3c.py:129-130), restated by hand
# ----------------------------------------------------------------------------

def ff_backward(params, x, acts, dlogits, dv, arch=ARCH_FF, dev_acts=None, mag=None):
    """Gradients of sum_i (dlogits_i . z_i + dv_i * v_i) for the A3CFF graph
    (a3c_ale.py:38-40) over a batch of samples.  acts = (a1, a2, h), or
    (a1, a2, a3, h) for the Nature head.  dev_acts: the HIP path's (a1, a2,
    h) for tie-aware ReLU masks (relu_mask)."""
    h = acts[-1]
    g = {}
    g["1/0/W"] = gmm(dlogits.T, h)
    g["1/0/b"] = gsum(dlogits)
    g["2/0/W"] = gmm(dv[None, :], h)
    g["2/0/b"] = gsum(dv[:, None])
    if mag is not None:
        mag["1/0/W"], mag["2/0/W"] = _mag_mm(dlogits.T, h), _mag_mm(dv[None, :], h)
        mag["1/0/b"], mag["2/0/b"] = _mag_sum(dlogits), _mag_sum(dv[:, None])
    dh = dlogits @ params["1/0/W"] + dv[:, None] * params["2/0/W"]
    if arch == ARCH_FF_NATURE:
        _nature_backward(params, x, acts, dh.astype(np.float32), g)
    else:
        a1, a2, _ = acts
        _head_backward(params, arch, x, a1, a2, h, dh.astype(np.float32), g, dev_acts, mag)
    return g


def _nature_backward(params, x, acts, dh, g):
    """Backward of NatureDQNHead (dqn_head.py:24-28) from dL/dh."""
    arch = ARCH_FF_NATURE
    a1, a2, a3, h = acts
    n = x.shape[0]
    dfc = dh * (h > 0)
    g[pname(arch, "fcW")] = gmm(dfc.T, a3.reshape(n, -1))
    g[pname(arch, "fcb")] = gsum(dfc)
    da3 = ((dfc @ params[pname(arch, "fcW")]).reshape(a3.shape) * (a3 > 0)).astype(np.float32)
    gW3, gb3, da2 = conv2d_backward(a2, params[pname(arch, "c3W")], da3, 1)
    g[pname(arch, "c3W")], g[pname(arch, "c3b")] = gW3, gb3
    da2 = (da2 * (a2 > 0)).astype(np.float32)
    gW2, gb2, da1 = conv2d_backward(a1, params[pname(arch, "c2W")], da2, 2)
    g[pname(arch, "c2W")], g[pname(arch, "c2b")] = gW2, gb2
    da1 = (da1 * (a1 > 0)).astype(np.float32)
    gW1, gb1, _ = conv2d_backward(x, params[pname(arch, "c1W")], da1, 4, need_dx=False)
    g[pname(arch, "c1W")], g[pname(arch, "c1b")] = gW1, gb1


def relu_mask(a, a_dev=None, rel=1e-5):
    """ReLU gradient mask a > 0.  Tie-aware with a_dev (the HIP path's own
    post-ReLU activations): where both are below rel * max|a| -- a
    pre-activation within rounding of 0, where either sign is a correct f32
    result -- the HIP path's decision is taken, so a parity test compares
    the arithmetic rather than a coin flip at a tie."""
    m = a > 0
    if a_dev is None:
        return m
    a_dev = np.asarray(a_dev, np.float32).reshape(a.shape)
    eps = F32(rel) * max(float(np.abs(a).max()), 1e-30)
    tie = (a < eps) & (a_dev < eps)
    return np.where(tie, a_dev > 0, m)


def _mag_mm(a, b):
    """Error scale of each element of the reduction a @ b (a = x^T, M x S;
    b = y, S x N): sqrt(sum_s (|x_si| Y + X |y_sj|)^2), X and Y the largest
    |x| and |y|.  An f32 operand value carries an absolute rounding error of
    order eps * (its tensor's largest value) -- a pre-activation summed from
    many terms, an advantage R - v, a near-zero ReLU output -- so a summand
    x y is uncertain by about |x| dY + |y| dX; the element's error is that
    summed in quadrature.  Tests hold |gpu - oracle| <= rtol * scale."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    X = float(np.abs(a).max()) if a.size else 0.0
    Y = float(np.abs(b).max()) if b.size else 0.0
    sq = (Y * Y) * (a * a).sum(1)[:, None] + 2.0 * X * Y * (np.abs(a) @ np.abs(b)) + (X * X) * (b * b).sum(0)[None, :]
    return np.sqrt(sq)


def _mag_sum(a):
    """Error scale of a bias gradient (column sums of a, S x M): the summands'
    own uncertainty X per term in quadrature, X sqrt(S) (the "ones" operand
    is exact)."""
    a = np.asarray(a, np.float64)
    X = float(np.abs(a).max()) if a.size else 0.0
    return np.full(a.shape[1], X * np.sqrt(a.shape[0]))


def _head_backward(params, arch, x, a1, a2, h, dh, g, dev_acts=None, mag=None):
    n = x.shape[0]
    d1, d2, dhh = dev_acts if dev_acts is not None else (None, None, None)
    dfc = dh * relu_mask(h, dhh)
    g[pname(arch, "fcW")] = gmm(dfc.T, a2.reshape(n, -1))
    g[pname(arch, "fcb")] = gsum(dfc)
    if mag is not None:
        mag[pname(arch, "fcW")] = _mag_mm(dfc.T, a2.reshape(n, -1))
        mag[pname(arch, "fcb")] = _mag_sum(dfc)
    da2 = (dfc @ params[pname(arch, "fcW")]).reshape(a2.shape) * relu_mask(a2, d2)
    gW2, gb2, da1 = conv2d_backward(a1, params[pname(arch, "c2W")],
                                    da2.astype(np.float32), 2, mag=mag,
                                    names=(pname(arch, "c2W"), pname(arch, "c2b")))
    g[pname(arch, "c2W")], g[pname(arch, "c2b")] = gW2, gb2
    da1 = (da1 * relu_mask(a1, d1)).astype(np.float32)
    gW1, gb1, _ = conv2d_backward(x, params[pname(arch, "c1W")], da1, 4,
                                  need_dx=False, mag=mag,
                                  names=(pname(arch, "c1W"), pname(arch, "c1b")))
    g[pname(arch, "c1W")], g[pname(arch, "c1b")] = gW1, gb1


# ----------------------------------------------------------------------------
# GradientClipping(40) (a3c_ale.py:226, Chainer hook) and RMSpropAsync
# ----------------------------------------------------------------------------

def grad_sqnorm(grads) -> float:
    """Chainer _sum_sqnorm: per-array f32 dot, summed as Python floats."""
    return float(sum(float(np.dot(gv.ravel(), gv.ravel())) for gv in grads))


def clip_grads(grads, threshold=40.0, exact_norm=False):
    """GradientClipping: rate = threshold / norm; if rate < 1: g *= rate
    (f32 array *= f64 scalar -> f32 multiply by f32(rate)).  exact_norm:
    accumulate the squared norm in f64 instead of Chainer's per-array f32
    dot (whose own rounding is ~sqrt(n) ulp on 677k-element arrays)."""
    if exact_norm:
        norm = math.sqrt(sum(float((gv.astype(np.float64) ** 2).sum()) for gv in grads))
    else:
        norm = math.sqrt(grad_sqnorm(grads))
    rate = threshold / norm if norm > 0 else float("inf")
    if rate < 1:
        r32 = F32(rate)
        return [(gv * r32).astype(np.float32) for gv in grads], norm
    return [gv.copy() for gv in grads], norm


def rmsprop_update(p, ms, g, lr, alpha=0.99, eps=0.1):
    """rmsprop_async.py:23-29 (update_one_cpu), f32 rounding of each op:
    ms *= alpha; ms += (1-alpha)*g*g; p -= lr*g/sqrt(ms+eps)."""
    p = p.astype(np.float32).copy()
    ms = ms.astype(np.float32).copy()
    ms *= F32(alpha)
    ms += (F32(1 - alpha) * g) * g
    p -= (F32(lr) * g) / np.sqrt(ms + F32(eps))
    return p, ms


def annealed_lr(lr0, total_steps, global_t):
    """a3c_ale.py:111-112."""
    return (total_steps - global_t - 1) / total_steps * lr0


# ----------------------------------------------------------------------------
# Lockstep window (batched A3C): per-env segments at fixed theta
# ----------------------------------------------------------------------------

def state_from_ring(frames, nvalid, slots):
    """Build (N,4,84,84) f32 states from ring planes frames[slot] (N,84,84)
    for the 4 slots oldest->newest, zeroing planes before the last reset
    (nvalid in 1..4 = number of valid trailing planes)."""
    n = nvalid.shape[0]
    x = np.zeros((n, 4, DST, DST), np.float32)
    for c in range(4):
        pl = PHI_LUT[frames[slots[c]]]
        keep = (c >= 4 - nvalid.astype(np.int32))
        x[:, c] = np.where(keep[:, None, None], pl, F32(0.0))
    return x


@dataclass
class LSTMState:
    h: np.ndarray
    c: np.ndarray
    has: np.ndarray   # (N,) bool


def ff_window_grads(params, states, actions, rewards, dones, boot_state,
                    gamma=0.99, beta=0.01, v_loss_coef=0.5, arch=ARCH_FF, dev_acts=None, **loss_kw):
    """Gradient of one lockstep window for A3CFF at fixed theta.

    states: (T, N, 4, 84, 84) f32; boot_state (N,4,84,84) f32 = s_T.
    Per env the window splits into segments at terminals; each segment is
    one a3c.py:77-130 update at fixed theta; gradients are summed."""
    T, N = actions.shape
    x = states.reshape(T * N, states.shape[2], DST, DST)   # 4 planes, or 3 for ARCH_RGB
    logits, v, acts = pi_and_v_ff(params, x, arch)
    p = softmax(logits)
    lp = log_softmax(logits)
    _, vb, _ = pi_and_v_ff(params, boot_state, arch)
    A = logits.shape[1]
    R, adv, dlog, dv, pil, vl = returns_and_lossgrad(
        rewards, dones, v.reshape(T, N), vb, p.reshape(T, N, A),
        lp.reshape(T, N, A), actions, gamma, beta, v_loss_coef, **loss_kw)
    mag = {} if arch != ARCH_FF_NATURE else None
    g = ff_backward(params, x, acts, dlog.reshape(T * N, A), dv.reshape(T * N), arch, dev_acts, mag)
    return g, dict(logits=logits.reshape(T, N, A), v=v.reshape(T, N), vboot=vb,
                   R=R, adv=adv, dlogits=dlog, dv=dv, pi_loss=pil, v_loss=vl, grad_mag=mag)


def lstm_window(params, states, actions, rewards, dones_prev, dones, boot_state,
                st0: LSTMState, gamma=0.99, beta=0.01, v_loss_coef=0.5, dev_acts=None, **loss_kw):
    """A3CLSTM window (a3c_ale.py:55-70) at fixed theta with truncated BPTT
    over the window (unchain_backward, a3c.py:144) and resets at terminals.

    dones_prev: (T, N): reset before step t (done of transition t-1 -> t;
    row 0 = the flag carried from the previous window)."""
    T, N = actions.shape
    arch = ARCH_LSTM
    A = params["2/0/W"].shape[0]
    xs = states.reshape(T * N, states.shape[2], DST, DST)
    a1, a2, hh = nips_head(params, arch, xs)
    hh = hh.reshape(T, N, 256)
    hs, cs, gs, has_l, hprev_l, cprev_l = [], [], [], [], [], []
    h, c, has = st0.h, st0.c, st0.has.copy()
    for t in range(T):
        has = has & (dones_prev[t] == 0)
        g, c_new, h_new = lstm_cell(params, arch, hh[t], h, c, has)
        hprev_l.append(h * has[:, None]); cprev_l.append(c * has[:, None])
        has_l.append(has.copy()); gs.append(g)
        h, c = h_new, c_new
        has = np.ones(N, bool)
        hs.append(h); cs.append(c)
    H = np.stack(hs)
    logits = linear(H.reshape(T * N, 256), params["2/0/W"], params["2/0/b"])
    v = linear(H.reshape(T * N, 256), params["3/0/W"], params["3/0/b"])[:, 0]
    p = softmax(logits); lp = log_softmax(logits)
    # bootstrap with keep_same_state (a3c_ale.py:57-60)
    _, _, hb = nips_head(params, arch, boot_state)
    hasb = has & (dones[T - 1] == 0)
    _, _, hbb = lstm_cell(params, arch, hb, h, c, hasb)
    vb = linear(hbb, params["3/0/W"], params["3/0/b"])[:, 0]
    R, adv, dlog, dv, pil, vl = returns_and_lossgrad(
        rewards, dones, v.reshape(T, N), vb, p.reshape(T, N, A),
        lp.reshape(T, N, A), actions, gamma, beta, v_loss_coef, **loss_kw)
    dl = dlog.reshape(T * N, A); dvf = dv.reshape(T * N)
    g = {}
    Hf = H.reshape(T * N, 256)
    g["2/0/W"] = gmm(dl.T, Hf)
    g["2/0/b"] = gsum(dl)
    g["3/0/W"] = gmm(dvf[None, :], Hf)
    g["3/0/b"] = gsum(dvf[:, None])
    mag = {"2/0/W": _mag_mm(dl.T, Hf), "3/0/W": _mag_mm(dvf[None, :], Hf),
           "2/0/b": _mag_sum(dl), "3/0/b": _mag_sum(dvf[:, None])}
    dH = (dl @ params["2/0/W"] + dvf[:, None] * params["3/0/W"]).reshape(T, N, 256)
    dh_next = np.zeros((N, 256), np.float32)
    dc_next = np.zeros((N, 256), np.float32)
    dG = np.zeros((T, N, 1024), np.float32)
    for t in reversed(range(T)):
        gt = gs[t]
        a = np.tanh(gt[:, 0::4]); i = sigmoid(gt[:, 1::4])
        f = sigmoid(gt[:, 2::4]); o = sigmoid(gt[:, 3::4])
        ct = cs[t]; tc = np.tanh(ct)
        dh = dH[t] + dh_next
        dc = dh * o * (F32(1) - tc * tc) + dc_next
        dg = np.zeros((N, 1024), np.float32)
        dg[:, 0::4] = dc * i * (F32(1) - a * a)
        dg[:, 1::4] = dc * a * i * (F32(1) - i)
        dg[:, 2::4] = dc * cprev_l[t] * f * (F32(1) - f)
        dg[:, 3::4] = dh * tc * o * (F32(1) - o)
        dG[t] = dg
        m = has_l[t].astype(np.float32)[:, None]
        dc_next = (dc * f * m).astype(np.float32)
        dh_next = ((dg @ params["1/lateral/W"]) * m).astype(np.float32)
    dGf = dG.reshape(T * N, 1024)
    g["1/upward/W"] = gmm(dGf.T, hh.reshape(T * N, 256))
    g["1/upward/b"] = gsum(dGf)
    g["1/lateral/W"] = gmm(dGf.T, np.stack(hprev_l).reshape(T * N, 256))
    mag["1/upward/W"] = _mag_mm(dGf.T, hh.reshape(T * N, 256))
    mag["1/upward/b"] = _mag_sum(dGf)
    mag["1/lateral/W"] = _mag_mm(dGf.T, np.stack(hprev_l).reshape(T * N, 256))
    dx = (dGf @ params["1/upward/W"]).astype(np.float32)
    _head_backward(params, arch, xs, a1, a2, hh.reshape(T * N, 256), dx, g, dev_acts, mag)
    aux = dict(logits=logits.reshape(T, N, A), v=v.reshape(T, N), vboot=vb,
               R=R, adv=adv, dlogits=dlog, dv=dv, pi_loss=pil, v_loss=vl,
               h_last=h, c_last=c, has_last=has, grad_mag=mag)
    return g, aux


def flat_names(arch, n_actions):
    return [n for n, _ in param_shapes(arch, n_actions)]


# ----------------------------------------------------------------------------
# The reference's one-env agent: a3c.py:27-167 (A3C.act) driven call by call,
# with GradientClipping + RMSpropAsync (a3c_ale.py:224-226) after each update
# ----------------------------------------------------------------------------

class A3CAgent:
    """a3c.py:67-167 for one env (one reference process) on the oracle's
    math.  act() mirrors the reference's control flow: the window restarts at
    every update (t_start = t, a3c.py:152), a terminal call runs the R = 0
    update and returns None (a3c.py:77-83,165-167), a full window
    bootstraps from v(s) at the pre-update parameters and then acts on s with
    the post-update ones (a3c.py:85,156).  Actions are drawn by inverse CDF
    from Philox(seed; env 0, t_max * updates + step in window), or taken from
    `action` when given.  Records per call and per update are appended to
    self.calls / self.updates."""

    def __init__(self, params, arch, n_actions, t_max=5, gamma=0.99, beta=0.01, pi_loss_coef=1.0,
                 v_loss_coef=0.5, keep_loss_scale_same=False, clip=40.0, seed=0, clip_reward=True, phi=None):
        self.p = {k: np.asarray(v, np.float32).copy() for k, v in params.items()}
        self.ms = {k: np.zeros_like(v) for k, v in self.p.items()}
        self.arch, self.A, self.T = arch, n_actions, t_max
        self.gamma, self.beta, self.clip, self.seed = gamma, beta, clip, seed
        self.clip_reward = clip_reward
        self.phi = phi                    # None: dqn_phi (a3c_ale.py:220); else the model sees phi(state)
        self.loss_kw = dict(pi_loss_coef=pi_loss_coef, keep_loss_scale_same=keep_loss_scale_same, t_max=t_max)
        self.v_loss_coef = v_loss_coef
        self.t = self.t_start = 0
        self.n_upd = 0
        self.rewards = {}
        self.win_x, self.win_a = [], []
        self.names = flat_names(arch, n_actions)
        # LSTM: recurrent state after the latest step (None -> has = False)
        self.h = np.zeros((1, 256), np.float32)
        self.c = np.zeros((1, 256), np.float32)
        self.has = False
        self.win_st0 = None
        self.calls, self.updates = [], []

    def _forward(self, x, h, c, has):
        a1, a2, hfc = nips_head(self.p, self.arch, x)
        c2 = h2 = None
        if self.arch == ARCH_LSTM:
            _, c2, h2 = lstm_cell(self.p, self.arch, hfc, h, c, np.array([has]))
            hfc = h2
        w = "2/0" if self.arch == ARCH_LSTM else "1/0"
        vw = "3/0" if self.arch == ARCH_LSTM else "2/0"
        logits = linear(hfc, self.p[w + "/W"], self.p[w + "/b"])
        v = linear(hfc, self.p[vw + "/W"], self.p[vw + "/b"])[:, 0]
        return logits, v, c2, h2

    def act(self, screens, reward, terminal, lr, action=None):
        T = self.T
        if self.clip_reward:
            reward = float(np.clip(reward, -1, 1))            # a3c.py:69-70
        if terminal:
            x = None
        elif self.phi is None:
            x = PHI_LUT[np.asarray(screens, np.uint8)][None]
        else:
            x = np.asarray(self.phi(screens), np.float32)[None]   # a3c.py:73
        self.rewards[self.t - 1] = reward                     # a3c.py:75
        if (terminal and self.t_start < self.t) or self.t - self.t_start == T:
            self._update(x, terminal, lr)
        if terminal:                                          # a3c.py:165-167
            self.has = False
            self.calls.append(None)
            return None
        logits, v, c2, h2 = self._forward(x, self.h, self.c, self.has)
        p, lp = softmax(logits), log_softmax(logits)
        if action is None:
            u = sample_uniforms(self.seed, np.array([0]), T * self.n_upd + (self.t - self.t_start))
            action = int(sample_from_uniform(p, u)[0])
        if self.t == self.t_start:
            self.win_st0 = LSTMState(self.h.copy(), self.c.copy(), np.array([self.has]))
        if self.arch == ARCH_LSTM:
            self.h, self.c, self.has = h2, c2, True
        self.win_x.append(x[0])
        self.win_a.append(action)
        self.t += 1
        self.calls.append(dict(action=action, probs=p[0], v=float(v[0]), entropy=float(entropy(p, lp)[0])))
        return action

    def _update(self, x, terminal, lr):
        L = self.t - self.t_start
        states = np.stack(self.win_x)[:, None]
        acts = np.array(self.win_a, np.int32)[:, None]
        r = np.array([[self.rewards[i]] for i in range(self.t_start, self.t)], np.float32)
        d = np.zeros((L, 1), np.uint8)
        if terminal:
            d[L - 1] = 1
        boot = states[-1] if terminal else x
        kw = dict(gamma=self.gamma, beta=self.beta, v_loss_coef=self.v_loss_coef, **self.loss_kw)
        if self.arch == ARCH_LSTM:
            dprev = np.zeros((L, 1), np.uint8)
            g, aux = lstm_window(self.p, states, acts, r, dprev, d, boot, self.win_st0, **kw)
        else:
            g, aux = ff_window_grads(self.p, states, acts, r, d, boot, **kw)
        grads = [g[n] for n in self.names]
        clipped, norm = clip_grads(grads, self.clip)
        for n, gc in zip(self.names, clipped):
            self.p[n], self.ms[n] = rmsprop_update(self.p[n], self.ms[n], gc, lr)
        self.updates.append(dict(call=len(self.calls), L=L, terminal=terminal, R=aux["R"][:, 0].copy(),
                                 v=aux["v"][:, 0].copy(), pi_loss=aux["pi_loss"], v_loss=aux["v_loss"],
                                 grads=dict(g), norm=norm, params={n: self.p[n].copy() for n in self.names}))
        self.n_upd += 1
        self.t_start = self.t                                 # a3c.py:152
        self.rewards = {}
        self.win_x, self.win_a = [], []
