"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference-generated golden fixtures.

Tolerances (stated per test): integer / byte / index work is bit-exact;
fp32 contractions |gpu - oracle| <= 1e-5 * max(|oracle|, ||oracle||_inf)
(norm-scaled); the RMSProp kernel is bit-exact vs the reference."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from conftest import close_normscaled, golden, grads_match, load_checkpoint
from sim import OracleEnvView, OracleRgbView, OracleStatesView, make_pools, make_rgb_pools, make_state_pools

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def dev(x, gpu):
    return torch.from_numpy(np.ascontiguousarray(x)).to(gpu)


# ------------------------------------------------------------------ phi
def test_luminance_all_rgb_triples(gpu):
    from asyncrl_amd import max_luminance
    trip = np.arange(1 << 24, dtype=np.uint32)
    rgb = np.stack([(trip >> 16) & 255, (trip >> 8) & 255, trip & 255], -1).astype(np.uint8)
    zero = np.zeros_like(rgb)
    g = max_luminance(dev(rgb, gpu), dev(zero, gpu)).cpu().numpy()
    assert (g == O.luminance_u8(rgb)).all()
    # max() of the pair: swap roles with a shifted copy
    other = np.roll(rgb, 12345, axis=0)
    g2 = max_luminance(dev(other, gpu), dev(rgb, gpu)).cpu().numpy()
    assert (g2 == O.luminance_u8(np.maximum(rgb, other))).all()


def test_current_screen_matches_reference_golden(gpu):
    from asyncrl_amd import current_screen
    d = golden("phi_golden.npz")
    cur, prev = dev(d["cur"], gpu), dev(d["prev"], gpu)
    out = current_screen(cur, prev, 0).cpu().numpy()
    assert (out == d["screen_scalar"]).all()
    simd = current_screen(cur, prev, 1).cpu().numpy()
    ref = np.stack([O.current_screen(c, p, O.RESIZE_SIMD) for c, p in zip(d["cur"], d["prev"])])
    assert (simd == ref).all()
    # ale.py:73-82 crop branch (RESIZE_CROP flag), both vertical-pass forms
    crop = current_screen(cur, prev, O.RESIZE_CROP).cpu().numpy()
    assert (crop == golden("phi_crop_golden.npz")["screen_crop"]).all()
    crop_simd = current_screen(cur, prev, O.RESIZE_CROP | O.RESIZE_SIMD).cpu().numpy()
    ref = np.stack([O.current_screen(c, p, O.RESIZE_CROP | O.RESIZE_SIMD) for c, p in zip(d["cur"], d["prev"])])
    assert (crop_simd == ref).all()


@pytest.mark.parametrize("kind,mode", [("uniform", 0), ("palette", 0), ("uniform", 2), ("palette", 3)])
def test_phi_stack_matches_oracle(gpu, kind, mode):
    from asyncrl_amd import phi_stack
    rng = np.random.default_rng(11)
    n = 37
    pairs, _, _ = make_pools(rng, 1, n, kind)
    pairs = pairs[0]
    prev = rng.integers(0, 256, (n, 4, 84, 84), dtype=np.uint8)
    reset = (rng.random(n) < 0.3).astype(np.uint8)
    out = phi_stack(dev(pairs, gpu), dev(prev, gpu), dev(reset, gpu), resize_mode=mode).cpu().numpy()
    for e in range(n):
        scr = O.current_screen(pairs[e, 0], pairs[e, 1], mode)
        assert (out[e] == O.stack_push(prev[e], scr, bool(reset[e]))).all(), e


@pytest.mark.parametrize("H,W", [(480, 640), (240, 320), (120, 160)])
def test_rgb_phi_matches_oracle(gpu, H, W):
    """train_a3c_doom.py:21-23 batched (arl_rgb_phi) on the three
    doom_env.py resolutions, both vertical-pass forms: bit-exact f32."""
    from asyncrl_amd import rgb_phi
    rng = np.random.default_rng(W)
    n = 6
    imgs = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    imgs[0] = 255
    imgs[1] = 0
    imgs[2, :, :W // 2] = rng.integers(0, 256, 3, dtype=np.uint8)   # flat blocks + edges
    d = dev(imgs, gpu)
    for mode in (O.RESIZE_SCALAR, O.RESIZE_SIMD):
        out = rgb_phi(d, mode).cpu().numpy()
        for e in range(n):
            assert (out[e] == O.rgb_phi(imgs[e], mode)).all(), (mode, e)
    one = rgb_phi(d[3]).cpu().numpy()
    assert (one == O.rgb_phi(imgs[3])).all()


def test_dqn_phi_matches_reference_golden(gpu):
    from asyncrl_amd import dqn_phi
    d = golden("dqn_phi_golden.npz")
    out = dqn_phi(dev(d["stacks"], gpu)).cpu().numpy()
    assert (out == d["out"]).all()
    allv = np.tile(np.arange(256, dtype=np.uint8), 4 * 84 * 84 // 256 + 1)[:4 * 84 * 84].reshape(1, 4, 84, 84)
    assert (dqn_phi(dev(allv, gpu)).cpu().numpy() == O.PHI_LUT[allv]).all()


def test_observe_ring_reproduces_reference_stacks(gpu):
    """arl_observe over 12 steps with resets: the ring + nvalid view equals
    the ale.py deque semantics (oracle.stack_push) at every step."""
    from asyncrl_amd import DeviceNet
    rng = np.random.default_rng(12)
    N, T, P = 5, 5, 12
    pairs, rewards, dones = make_pools(rng, P, N, "palette", p_done=0.25)
    net = DeviceNet(0, 4, N, T)
    net.reset()
    view = OracleEnvView(pairs, dones)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    frames = net.buffer("frames", torch.uint8, (net.t_max + 4, N, 84, 84))
    nvalid = net.buffer("nvalid", torch.uint8, (net.t_max + 4, N))
    R = T + 4
    rew = net.buffer("rewards", torch.float32, (T, N))
    dn = net.buffer("dones", torch.uint8, (T, N))
    for w in range(2):                      # obs steps k = w*T + t
        for t in range(0 if w == 0 else 1, T + 1):
            k = w * T + t
            net.observe(t, dp, dr, dd, P, force_reset=(k == 0))
            fr, nv = frames.cpu().numpy(), nvalid.cpu().numpy()
            want = view.stack(k)
            for e in range(N):
                got = np.stack([fr[(k - 3 + c) % R, e] if c >= 4 - nv[k % R, e]
                                else np.zeros((84, 84), np.uint8) for c in range(4)])
                assert (got == want[e]).all(), (k, e)
            if t >= 1:   # reward / done of the transition into obs k
                assert (rew[t - 1].cpu().numpy() == rewards[k % P]).all()
                assert (dn[t - 1].cpu().numpy() == dones[k % P]).all()
        net.advance()


# ------------------------------------------------------------------ forward / policy
def test_forward_real_checkpoint_matches_oracle(gpu):
    from asyncrl_amd import A3CFF, dqn_phi
    ck = load_checkpoint()
    n = 24
    model = A3CFF(4, n_envs=n, t_max=5, init_seed=None)
    model.net.load_params(ck)
    rng = np.random.default_rng(13)
    stacks = rng.integers(0, 256, (n, 4, 84, 84), dtype=np.uint8)
    stacks[:4, :2] = 0
    x = dqn_phi(dev(stacks, gpu))
    pout, v = model.pi_and_v(x)
    lo, vo, _ = O.pi_and_v_ff(ck, O.PHI_LUT[stacks])
    for got, want in ((pout.logits, lo), (v, vo), (pout.probs, O.softmax(lo)),
                      (pout.log_probs, O.log_softmax(lo))):
        ok, err = close_normscaled(got.cpu().numpy(), want, RTOL)
        assert ok, err
    ent = O.entropy(O.softmax(lo), O.log_softmax(lo))
    assert close_normscaled(pout.entropy.cpu().numpy(), ent, RTOL)[0]


def _heads(rng, A):
    b = 1.0 / np.sqrt(256)
    W_pi = rng.uniform(-b, b, (A, 256)).astype(np.float32)
    b_pi = rng.uniform(-b, b, A).astype(np.float32)
    W_v = rng.uniform(-b, b, (1, 256)).astype(np.float32)
    b_v = rng.uniform(-b, b, 1).astype(np.float32)
    return W_pi, b_pi, W_v, b_v


@pytest.mark.parametrize("A", [4, 6, 18, 32])
def test_policy_heads_and_sampling_match_oracle(gpu, A):
    """arl_policy: logits / probs / log_probs / v / entropy within RTOL of the
    oracle, and the sampled actions bit-exact given the same Philox uniforms
    (oracle.sample_uniforms + inverse CDF over the kernel's own probs)."""
    from asyncrl_amd import fc_softmax_policy_and_v
    rng = np.random.default_rng(100 + A)
    n = 333
    h = np.maximum(rng.normal(0, 1, (n, 256)), 0).astype(np.float32) * 3
    W_pi, b_pi, W_v, b_v = _heads(rng, A)
    step = torch.tensor([41], dtype=torch.int64, device=gpu)
    pout, v = fc_softmax_policy_and_v(dev(h, gpu), dev(W_pi, gpu), dev(b_pi, gpu), dev(W_v, gpu), dev(b_v, gpu),
                                      seed=7, step=step, step_offset=2, env_offset=1000, mode=1)
    lo = h @ W_pi.T + b_pi
    vo = (h @ W_v.T + b_v)[:, 0]
    p_o, lp_o = O.softmax(lo), O.log_softmax(lo)
    for got, want in ((pout.logits, lo), (v, vo), (pout.probs, p_o), (pout.log_probs, lp_o),
                      (pout.entropy, O.entropy(p_o, lp_o))):
        ok, err = close_normscaled(got.cpu().numpy(), want, RTOL)
        assert ok, err
    probs = pout.probs.cpu().numpy()
    u = O.sample_uniforms(7, np.arange(1000, 1000 + n), 43)
    want_a = O.sample_from_uniform(probs, u)
    got_a = pout.action_indices.cpu().numpy()
    assert (got_a == want_a).all()
    lpa = pout.sampled_actions_log_probs.cpu().numpy()
    assert (lpa == pout.log_probs.cpu().numpy()[np.arange(n), got_a]).all()


def test_policy_sampling_frequencies_chi2(gpu):
    """Distributional parity with np.random.multinomial(1, p)
    (policy_output.py:12-29): 200k draws of one row (independent Philox
    streams per env id), chi-square goodness of fit against the probs."""
    from scipy.stats import chisquare
    from asyncrl_amd import fc_softmax_policy_and_v
    rng = np.random.default_rng(5)
    A, n = 6, 200_000
    h1 = np.maximum(rng.normal(0, 1, 256), 0).astype(np.float32) * 4
    W_pi, b_pi, W_v, b_v = _heads(rng, A)
    h = np.broadcast_to(h1, (n, 256)).copy()
    step = torch.tensor([3], dtype=torch.int64, device=gpu)
    pout, _ = fc_softmax_policy_and_v(dev(h, gpu), dev(W_pi, gpu), dev(b_pi, gpu), dev(W_v, gpu), dev(b_v, gpu),
                                      seed=11, step=step, mode=1)
    p = pout.probs[0].double().cpu().numpy()
    counts = np.bincount(pout.action_indices.cpu().numpy(), minlength=A)
    assert counts.sum() == n
    stat, pval = chisquare(counts, p / p.sum() * n)
    assert pval > 1e-4, (counts, p * n, pval)


def test_policy_greedy_most_probable_actions(gpu):
    """mode 2 = SoftmaxPolicyOutput.most_probable_actions (policy_output.py:37-39):
    the first argmax of the kernel's probs, through pi_and_v(deterministic=True)
    and through the standalone heads."""
    from asyncrl_amd import A3CFF, dqn_phi, fc_softmax_policy_and_v
    ck = load_checkpoint()
    n = 40
    model = A3CFF(4, n_envs=n, t_max=5, init_seed=None)
    model.net.load_params(ck)
    stacks = np.random.default_rng(21).integers(0, 256, (n, 4, 84, 84), dtype=np.uint8)
    pout, _ = model.pi_and_v(dqn_phi(dev(stacks, gpu)), deterministic=True)
    probs = pout.probs.cpu().numpy()
    assert (pout.most_probable_actions.cpu().numpy() == probs.argmax(1)).all()
    with pytest.raises(RuntimeError):
        pout.action_indices
    rng = np.random.default_rng(9)
    h = np.maximum(rng.normal(0, 1, (64, 256)), 0).astype(np.float32)
    W_pi, b_pi, W_v, b_v = _heads(rng, 7)
    W_pi[3] = W_pi[5]   # exact ties: the first index wins, as np.argmax
    b_pi[3] = b_pi[5]
    pout, _ = fc_softmax_policy_and_v(dev(h, gpu), dev(W_pi, gpu), dev(b_pi, gpu), dev(W_v, gpu), dev(b_v, gpu),
                                      mode=2)
    pr = pout.probs.cpu().numpy()
    assert (pout.most_probable_actions.cpu().numpy() == pr.argmax(1)).all()


# ------------------------------------------------------------------ full windows
def dev_acts(net, T, N):
    """The window's post-ReLU activations on the device (a1, a2, h) as the
    oracle's (T * N, ...) arrays, for its tie-aware ReLU masks."""
    a1 = net.buffer("a1", torch.float32, (T + 1, N, 16, 20, 20))[:T].cpu().numpy()
    a2 = net.buffer("a2", torch.float32, (T + 1, N, 32, 9, 9))[:T].cpu().numpy()
    h = net.buffer("hfc", torch.float32, (T + 1, N, 256))[:T].cpu().numpy()
    return a1.reshape(T * N, 16, 20, 20), a2.reshape(T * N, 32, 9, 9), h.reshape(T * N, 256)


def _grads_match(net, g_oracle, mag=None, rtol=RTOL):
    got = net.state_dict(net.grads)
    grads_match(got, g_oracle, mag, rtol)
    return got


def _run_ff(gpu, N, T, A, seed, kind, windows=2, ckpt=False, arch=O.ARCH_FF, p_done=None, hw=(120, 160)):
    from asyncrl_amd import A3C, A3CFF, A3CFFNature, DoomA3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(seed)
    P = 2 * T + 1
    rgb = bool(arch & O.ARCH_RGB)
    if kind == "states":
        pairs, rewards, dones = make_state_pools(rng, P, N, p_done=0.15 if p_done is None else p_done)
    elif rgb:
        pairs, rewards, dones = make_rgb_pools(rng, P, N, *hw, p_done=0.15 if p_done is None else p_done)
    else:
        pairs, rewards, dones = make_pools(rng, P, N, kind) if p_done is None else \
            make_pools(rng, P, N, kind, p_done=p_done)
    Model = A3CFFNature if arch == O.ARCH_FF_NATURE else (DoomA3CFF if rgb else A3CFF)
    model = Model(A, n_envs=N, t_max=T, seed=99, init_seed=seed, frames="states" if kind == "states" else "pairs")
    if ckpt:
        model.net.load_params(load_checkpoint())
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99)
    opt.setup(model)
    opt.add_hook(GradientClipping(40))
    agent = A3C(model, opt, T, 0.99, beta=1e-2)
    net = model.net
    view = OracleStatesView(pairs, dones) if kind == "states" else \
        OracleRgbView(pairs, dones) if rgb else OracleEnvView(pairs, dones)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    for w in range(windows):
        k0 = w * T
        params = net.state_dict()
        agent.run_window(dp, dr, dd, P, first=(w == 0), split_update=True)
        torch.cuda.synchronize()
        states, boot = view.states_f32(k0, T)
        r, d = view.window_rd(rewards, k0, T)
        acts = net.buffer("actions", torch.int32, (T + 1, N))[:T].cpu().numpy()
        g, aux = O.ff_window_grads(params, states, acts, r, d, boot, arch=arch,
                                   dev_acts=None if arch == O.ARCH_FF_NATURE else dev_acts(net, T, N))
        logits = net.buffer("logits", torch.float32, (T + 1, N, A))[:T].cpu().numpy()
        v = net.buffer("v", torch.float32, (T + 1, N)).cpu().numpy()
        assert close_normscaled(logits, aux["logits"], RTOL)[0]
        assert close_normscaled(v[:T], aux["v"], RTOL)[0]
        assert close_normscaled(v[T], aux["vboot"], RTOL)[0]
        dl = net.buffer("dlogits", torch.float32, (T, N, A)).cpu().numpy()
        assert close_normscaled(dl, aux["dlogits"], RTOL)[0]
        # sampling: exact given the GPU's probs and the oracle's Philox uniforms
        probs = net.buffer("probs", torch.float32, (T + 1, N, A)).cpu().numpy()
        for t in range(T):
            u = O.sample_uniforms(99, np.arange(N, dtype=np.uint64), k0 + t)
            assert (O.sample_from_uniform(probs[t], u) == acts[t]).all()
        got = _grads_match(net, g, aux["grad_mag"])
        # optimizer step: oracle clip + RMSProp applied to the device's own
        # gradient (already checked above at RTOL), compared as parameter deltas
        # (the clip rate's f64 vs per-array-f32 norm is the only difference)
        ms0 = net.state_dict(net.ms)
        agent.finish_window()
        torch.cuda.synchronize()
        names = list(g)
        gl, _ = O.clip_grads([got[k] for k in names], 40.0, exact_norm=True)
        new = net.state_dict()
        for k, gk in zip(names, gl):
            p1, _ = O.rmsprop_update(params[k], ms0[k], gk, 7e-4)
            ok, err = close_normscaled(new[k] - params[k], p1 - params[k], RTOL)
            assert ok, (k, err)


def test_ff_windows_match_oracle(gpu):
    _run_ff(gpu, N=6, T=5, A=4, seed=21, kind="uniform")


def test_ff_windows_real_checkpoint_palette_frames(gpu):
    _run_ff(gpu, N=5, T=5, A=4, seed=22, kind="palette", ckpt=True)


def test_ff_states_windows_match_oracle(gpu):
    """ARCH_STATES (the phi plugin's f32 state ring, generic-GEMM convs):
    signed float states that are no image of uint8 screens, 9 envs (ragged
    against the 64-row conv tiles), two windows with terminals."""
    _run_ff(gpu, N=9, T=5, A=4, seed=28, kind="states")


def test_ff_wide_action_set(gpu):
    _run_ff(gpu, N=3, T=3, A=18, seed=23, kind="uniform", windows=1)


# ------------------------------------------------------------------ edge cases
def test_ff_single_env_single_step_windows(gpu):
    """N = 1, t_max = 1 (every act is a window end: a3c.py:77-78 with
    t_max = 1), three windows: the smallest grid of every kernel."""
    _run_ff(gpu, N=1, T=1, A=4, seed=24, kind="uniform", windows=3)


def test_ff_ragged_env_count(gpu):
    """N = 67: one past the 64-env tiles, 3 past the 16-env policy rows and
    the 32-env FC tiles; two windows with terminals."""
    _run_ff(gpu, N=67, T=2, A=5, seed=25, kind="palette")


def test_ff_every_step_terminal(gpu):
    """Every observation ends an episode (done = 1 everywhere): every window
    segment has length 1 with R = 0 (a3c.py:82-83) and the stack resets every
    step (ale.py:155-158)."""
    _run_ff(gpu, N=4, T=3, A=4, seed=26, kind="uniform", p_done=1.0)


def test_ff_single_action(gpu):
    """A = 1: softmax = 1, entropy = 0, the sampler must return action 0."""
    _run_ff(gpu, N=5, T=3, A=1, seed=27, kind="uniform", windows=1)


def test_phi_entry_points_accept_empty_batches(gpu):
    """n = 0 is a no-op on every batched phi entry point (no launch, no error)."""
    from asyncrl_amd import current_screen, dqn_phi, phi_stack, rgb_phi
    z = torch.zeros((0, 210, 160, 3), dtype=torch.uint8, device=gpu)
    assert current_screen(z, z).shape == (0, 84, 84)
    zp = torch.zeros((0, 2, 210, 160, 3), dtype=torch.uint8, device=gpu)
    zs = torch.zeros((0, 4, 84, 84), dtype=torch.uint8, device=gpu)
    assert phi_stack(zp, zs).shape == (0, 4, 84, 84)
    assert dqn_phi(zs).shape == (0, 4, 84, 84)
    assert rgb_phi(torch.zeros((0, 480, 640, 3), dtype=torch.uint8, device=gpu)).shape == (0, 3, 84, 84)
    torch.cuda.synchronize()


def test_rgb_phi_rejects_unsupported_widths(gpu):
    """W must be a multiple of 16 (16-byte row loads) and <= 2048 (LDS);
    a bad shape fails loudly instead of reading out of bounds."""
    from asyncrl_amd import ArlError, rgb_phi
    with pytest.raises(ArlError):
        rgb_phi(torch.zeros((2, 100, 150, 3), dtype=torch.uint8, device=gpu))
    with pytest.raises(ArlError):
        rgb_phi(torch.zeros((1, 8, 4096, 3), dtype=torch.uint8, device=gpu))


def test_nature_head_windows_match_oracle(gpu):
    """Row a8: A3CFF with NatureDQNHead (dqn_head.py:6-28), two windows with
    terminals: forward, sampling, returns, every gradient tensor and the
    clip + RMSProp step against the oracle."""
    _run_ff(gpu, N=4, T=3, A=6, seed=41, kind="palette", arch=O.ARCH_FF_NATURE, p_done=0.2)


@pytest.mark.parametrize("hw", [(120, 160), (240, 320)])
def test_doom_ff_windows_match_oracle(gpu, hw):
    """train_a3c_doom.py:25-38 A3CFF on RGB screens (two doom_env.py
    resolutions): phi of the screen, the 3-channel NIPS head (fused kernels
    see [0, R, G, B]), sampling, returns, every gradient tensor (conv1 W
    (16, 3, 8, 8)) and the clip + RMSProp step against the oracle.  Seed 51
    puts a conv2 pre-activation within 1e-7 of 0, where the two summation
    orders disagree on the ReLU mask: the oracle's tie-aware masks
    (oracle.relu_mask) take the device's decision there."""
    _run_ff(gpu, N=5, T=4, A=3, seed=51, kind="uniform", arch=O.ARCH_FF | O.ARCH_RGB, p_done=0.2, hw=hw)


def test_doom_pi_and_v_matches_oracle(gpu):
    """DoomA3CFF.pi_and_v on rgb_phi states (drop-in for the Doom eval forward)."""
    from asyncrl_amd import DoomA3CFF, rgb_phi
    n, A = 19, 3
    model = DoomA3CFF(A, n_envs=n, t_max=5, init_seed=4)
    params = model.net.state_dict()
    imgs = np.random.default_rng(15).integers(0, 256, (n, 240, 320, 3), dtype=np.uint8)
    pout, v = model.pi_and_v(rgb_phi(dev(imgs, gpu)))
    x = np.stack([O.rgb_phi(i) for i in imgs])
    lo, vo, _ = O.pi_and_v_ff(params, x, O.ARCH_FF | O.ARCH_RGB)
    for got, want in ((pout.logits, lo), (v, vo), (pout.probs, O.softmax(lo))):
        ok, err = close_normscaled(got.cpu().numpy(), want, RTOL)
        assert ok, err


def test_nature_head_pi_and_v_matches_oracle(gpu):
    """A3CFFNature.pi_and_v on dqn_phi states (drop-in forward)."""
    from asyncrl_amd import A3CFFNature, dqn_phi
    n, A = 37, 4
    model = A3CFFNature(A, n_envs=n, t_max=5, init_seed=3)
    params = model.net.state_dict()
    stacks = np.random.default_rng(14).integers(0, 256, (n, 4, 84, 84), dtype=np.uint8)
    stacks[:5, :3] = 0
    pout, v = model.pi_and_v(dqn_phi(dev(stacks, gpu)))
    lo, vo, _ = O.pi_and_v_ff(params, O.PHI_LUT[stacks], O.ARCH_FF_NATURE)
    for got, want in ((pout.logits, lo), (v, vo), (pout.probs, O.softmax(lo))):
        ok, err = close_normscaled(got.cpu().numpy(), want, RTOL)
        assert ok, err


@pytest.mark.parametrize("rgb,N,T,A", [(False, 4, 5, 6), (True, 4, 5, 6), (False, 37, 2, 6), (False, 1, 1, 3)])
def test_lstm_windows_match_oracle(gpu, rgb, N, T, A):
    """A3CLSTM (a3c_ale.py:43-70) and, rgb=True, the ViZDoom A3CLSTM
    (train_a3c_doom.py:41-63) on 120 x 160 RGB screens; a ragged env count
    (37) and the N = 1, t_max = 1 corner."""
    from asyncrl_amd import A3C, A3CLSTM, DoomA3CLSTM, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(31)
    P = 2 * T + 1
    if rgb:
        pairs, rewards, dones = make_rgb_pools(rng, P, N, p_done=0.2)
    else:
        pairs, rewards, dones = make_pools(rng, P, N, "palette", p_done=0.2)
    model = (DoomA3CLSTM if rgb else A3CLSTM)(A, n_envs=N, t_max=T, seed=5, init_seed=31, frames="pairs")
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(GradientClipping(40))
    agent = A3C(model, opt, T, 0.99)
    net = model.net
    view = OracleRgbView(pairs, dones) if rgb else OracleEnvView(pairs, dones)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    st = O.LSTMState(h=np.zeros((N, 256), np.float32), c=np.zeros((N, 256), np.float32),
                     has=np.zeros(N, bool))
    prev_done = np.ones(N, np.uint8)
    for w in range(2):
        k0 = w * T
        params = net.state_dict()
        agent.run_window(dp, dr, dd, P, first=(w == 0), split_update=True)
        torch.cuda.synchronize()
        states, boot = view.states_f32(k0, T)
        r, d = view.window_rd(rewards, k0, T)
        dprev = np.concatenate([prev_done[None], d[:-1]], 0)
        acts = net.buffer("actions", torch.int32, (T + 1, N))[:T].cpu().numpy()
        g, aux = O.lstm_window(params, states, acts, r, dprev, d, boot, st, dev_acts=dev_acts(net, T, N))
        v = net.buffer("v", torch.float32, (T + 1, N)).cpu().numpy()
        assert close_normscaled(v[:T], aux["v"], RTOL)[0]
        assert close_normscaled(v[T], aux["vboot"], RTOL)[0]
        hb = net.buffer("hbuf", torch.float32, (T + 2, N, 256)).cpu().numpy()
        assert close_normscaled(hb[T], aux["h_last"], RTOL)[0]
        _grads_match(net, g, aux["grad_mag"])
        agent.finish_window()
        st = O.LSTMState(h=aux["h_last"], c=aux["c_last"], has=np.ones(N, bool))
        prev_done = d[-1]


def test_rmsprop_kernel_bitexact_vs_reference(gpu):
    from asyncrl_amd import RMSpropAsync
    r = golden("rmsprop_golden.npz")
    for k in range(r["p"].shape[0]):
        opt = RMSpropAsync(lr=float(r["lr"][k]), alpha=0.99, eps=0.1)
        p, ms, g = dev(r["p"][k], gpu), dev(r["ms"][k], gpu), dev(r["g"][k], gpu)
        opt.update_arrays(p, ms, g)
        assert (p.cpu().numpy() == r["p_out"][k]).all()
        assert (ms.cpu().numpy() == r["ms_out"][k]).all()


@pytest.mark.parametrize("n", [1, 2, 3, 5])
@pytest.mark.parametrize("clip", [False, True])
def test_rmsprop_tiny_arrays_match_oracle(gpu, n, clip):
    """update_one on arrays shorter than a float4 (the value-head bias has one
    element): no float4 pass, the tail handled element-wise; bit-exact with the
    oracle's f32 op sequence, the clip scale from the f64 norm."""
    from asyncrl_amd import GradientClipping, RMSpropAsync
    rng = np.random.default_rng(100 + n)
    p = rng.standard_normal(n).astype(np.float32)
    ms = np.abs(rng.standard_normal(n)).astype(np.float32) * 0.01
    g = (rng.uniform(1.0, 2.0, n) * rng.choice([-1.0, 1.0], n) * (60.0 if clip else 1.0)).astype(np.float32)
    opt = RMSpropAsync(lr=7e-4, alpha=0.99, eps=0.1)
    if clip:
        opt.add_hook(GradientClipping(40))
    P, M, G = dev(p, gpu), dev(ms, gpu), dev(g, gpu)
    opt.update_arrays(P, M, G)
    gc = g
    if clip:
        (gc,), norm = O.clip_grads([g], 40.0, exact_norm=True)
        assert norm > 40.0
    p1, m1 = O.rmsprop_update(p, ms, gc, 7e-4)
    if clip:   # the scale is one f32 rounding of the f64 norm on both sides
        assert np.allclose(P.cpu().numpy(), p1, rtol=1e-6, atol=1e-7)
        assert np.allclose(M.cpu().numpy(), m1, rtol=1e-6, atol=1e-9)
    else:
        assert (P.cpu().numpy() == p1).all() and (M.cpu().numpy() == m1).all()


def test_rmsprop_clip_matches_oracle(gpu):
    from asyncrl_amd import GradientClipping, RMSpropAsync
    rng = np.random.default_rng(41)
    n = 677429
    p = rng.standard_normal(n).astype(np.float32)
    ms = np.abs(rng.standard_normal(n)).astype(np.float32) * 0.01
    g = rng.standard_normal(n).astype(np.float32)
    opt = RMSpropAsync(lr=7e-4, alpha=0.99, eps=0.1)
    opt.add_hook(GradientClipping(40))
    P, M, G = dev(p, gpu), dev(ms, gpu), dev(g, gpu)
    opt.update_arrays(P, M, G)
    # f64-accumulated norm: NumPy's f32 dot (Chainer _sum_sqnorm) over 677k
    # elements is itself only ~1e-5 accurate; the kernel sums f32 partials
    # of ~10 elements in f64
    (gc,), norm = O.clip_grads([g], 40.0, exact_norm=True)
    p1, m1 = O.rmsprop_update(p, ms, gc, 7e-4)
    assert close_normscaled(P.cpu().numpy() - p, p1 - p, 1e-5)[0]
    assert close_normscaled(M.cpu().numpy(), m1, 1e-5)[0]


def test_graph_replay_equals_eager(gpu):
    """A captured window replays with advancing device step counters and
    gives bit-identical parameters to the eager path."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(51)
    N, T, P = 8, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform")
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)

    def mk():
        m = A3CFF(4, n_envs=N, t_max=T, seed=3, init_seed=4, frames="pairs")
        o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
        o.add_hook(GradientClipping(40))
        o.anneal_total_steps, o.n_total_envs = 10 ** 6, N
        return A3C(m, o, T, 0.99)

    a, b = mk(), mk()
    for w in range(4):
        a.run_window(dp, dr, dd, P, first=(w == 0))
    b.run_window(dp, dr, dd, P, first=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        b.run_window(dp, dr, dd, P, first=False)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a.net.params, b.net.params)
    assert torch.equal(a.net.ms, b.net.ms)


def test_many_windows_stay_finite(gpu):
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(61)
    N, T, P = 16, 5, 9
    pairs, rewards, dones = make_pools(rng, P, N, "palette")
    m = A3CFF(4, n_envs=N, t_max=T, seed=1, frames="pairs")
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
    o.add_hook(GradientClipping(40))
    agent = A3C(m, o, T, 0.99)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    for w in range(30):
        agent.run_window(dp, dr, dd, P, first=(w == 0))
    torch.cuda.synchronize()
    assert torch.isfinite(m.net.params).all()
    acts = m.net.buffer("actions", torch.int32, (T + 1, N))[:T]
    assert int(acts.min()) >= 0 and int(acts.max()) < 4


@pytest.mark.parametrize("arch,N,groups", [("ff", 96, 3), ("ff", 256, 2), ("lstm", 80, 2), ("doom_ff", 64, 2)])
def test_env_groups_identical(gpu, arch, N, groups):
    """run_window(env_groups=G): G forward chains on G streams (staggered by
    one kernel), eager and graph-captured, give bit-identical actions,
    values, gradients, parameters and RMSProp state to one chain."""
    from asyncrl_amd import A3C, A3CFF, A3CLSTM, DoomA3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(71)
    T, P = 5, 7
    Model = {"ff": A3CFF, "lstm": A3CLSTM, "doom_ff": DoomA3CFF}[arch]
    A = 3 if arch == "doom_ff" else 4
    if arch == "doom_ff":
        pairs = rng.integers(0, 256, size=(P, N, 120, 160, 3), dtype=np.uint8)
        rewards = rng.choice([-1.0, 0.0, 1.0], p=[0.05, 0.9, 0.05], size=(P, N)).astype(np.float32)
        dones = (rng.random((P, N)) < 0.1).astype(np.uint8)
    else:
        pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)

    def mk():
        m = Model(A, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs")
        o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
        o.add_hook(GradientClipping(40))
        o.anneal_total_steps, o.n_total_envs = 10 ** 6, N
        return A3C(m, o, T, 0.99)

    a, b = mk(), mk()
    assert len(b.net.env_groups(groups)) == groups
    outs = []
    for ag, G in ((a, 1), (b, groups)):
        ag.run_window(dp, dr, dd, P, first=True, env_groups=G)
        ag.run_window(dp, dr, dd, P, env_groups=G)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ag.run_window(dp, dr, dd, P, stream=s, env_groups=G)   # creates the side streams before capture
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            ag.run_window(dp, dr, dd, P, stream=s, env_groups=G, split_update=True)
        g.replay()
        torch.cuda.synchronize()
        net = ag.net
        outs.append({"actions": net.buffer("actions", torch.int32, (T + 1, N)).clone(),
                     "v": net.buffer("v", torch.float32, (T + 1, N)).clone(),
                     "grads": net.grads.clone(), "params": net.params.clone(), "ms": net.ms.clone()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("arch", ["ff", "lstm"])
def test_learn_parts_identical(gpu, arch):
    """arl_learn_part 0..2 in order on one stream (the N > 1 window's split
    learner) gives the same gradient bits as arl_learn in one call."""
    from asyncrl_amd import A3C, A3CFF, A3CLSTM, RMSpropAsync
    rng = np.random.default_rng(81)
    N, T, P = 48, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    Model = A3CFF if arch == "ff" else A3CLSTM
    m = Model(4, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs")
    ag = A3C(m, RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m), T, 0.99)
    ag.run_window(dp, dr, dd, P, first=True, split_update=True)
    net = ag.net
    got = []
    for parts in (False, True, False):
        net.grads.fill_(1234.5)            # padding between tensors keeps it
        if parts:
            net.learn_parts(range(3))
        else:
            net.learn()
        torch.cuda.synchronize()
        got.append(net.grads.clone())
    for name in net.layout:               # every tensor was written
        g = net.view(got[0], name)
        assert torch.isfinite(g).all() and not (g == 1234.5).any(), name
    assert torch.equal(got[0], got[1]) and torch.equal(got[0], got[2])


def test_lstm_fc_reduce_forms_identical(gpu, tmp_path):
    """LSTM windows (two env groups, eager and graph-captured) with the FC
    forward's split-K partials reduced in the gate kernel's staging (the
    default under 512 envs a launch) and by the FC's last-arriver ticket
    (ARL_LSTM_XRED=0): the same partials summed in the same order, so hidden /
    cell states, gates, actions, values, gradients and parameters match bit
    for bit."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    outs = []
    for extra in ({}, {"ARL_LSTM_XRED": "0"}):
        f = str(tmp_path / f"lstm_{len(outs)}.npz")
        env = dict(os.environ, **extra)
        subprocess.run([sys.executable, os.path.join(here, "lstm_split_worker.py"), f], env=env, check=True,
                       timeout=240)
        outs.append(np.load(f))
    assert int((outs[0]["hbuf"] != 0).sum()) > 0
    for o in outs[1:]:
        for k in outs[0].files:
            assert np.array_equal(outs[0][k], o[k]), k


def test_norm_fold_matches_grad_sqnorm(gpu):
    """The clip norm folded into the learner's conv reduce (one rank,
    arl_net_set_norm_fold) against the separate grad_sqnorm launch: the same
    gradient (bit-identical), and after clip + RMSProp parameters within 1e-6
    (the f64 partial sums group differently), with clipping active."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(17)
    N, T, P = 64, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    outs = []
    for fold in (False, True):
        m = A3CFF(4, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs")
        o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
        o.add_hook(GradientClipping(1.0))   # small threshold: clipping is active
        ag = A3C(m, o, T, 0.99)
        ag.net.set_norm_fold(fold)
        ag.run_window(dp, dr, dd, P, first=True)
        torch.cuda.synchronize()
        g = ag.net.grads.clone()                             # window 1's gradient (same parameters in both arms)
        for w in range(2):
            ag.run_window(dp, dr, dd, P)
        torch.cuda.synchronize()
        outs.append((g, ag.net.params.clone(), float(g.double().pow(2).sum().sqrt())))
    assert outs[0][2] > 1.0                                  # the clip was active
    assert torch.equal(outs[0][0], outs[1][0])               # same gradient bits
    ok, err = close_normscaled(outs[1][1].cpu().numpy(), outs[0][1].cpu().numpy(), 1e-6)
    assert ok, err


@pytest.mark.parametrize("n_envs", [1, 33, 75, 200, 512])
def test_conv_fwd_two_envs_identical(gpu, tmp_path, n_envs):
    """The large-launch forms against the 256-env ones: conv_fwd.hip with two
    envs a workgroup (EPW = 2: 16 waves sharing the weight planes) and fc.hip's
    64-row tiles (fc_fwd_big_kernel), the defaults from 512 envs a launch.  The
    per-tile k order is the same, so a1, a2, hfc, the policy outputs and
    actions, the window gradient and the updated parameters match bit for bit
    -- at an odd env count (the last conv workgroup's second slot idle, a
    partial FC tile), at 200 (a partial 64-row block) and at 512.  And the
    window as one C call (arl_run_window) against its launches issued step by
    step from Python (ARL_WINDOW_C=0): the C window runs the learner's returns
    and heads backward inside the bootstrap policy launch
    (policy_fc_returns_kernel), so dlogits / dv / the losses / dfc are compared
    too -- also at 1 and 33 envs; the last arm issues the window step by step
    with the fusion off (ARL_FUSE_RETURNS=0: the separate returns_heads_kernel
    launch), so the fused launch is checked bitwise against the unfused one.
    ARL_CB_WS=0: conv_bwd.hip's 512-thread kernel against the default
    wave-specialised one (1,024 threads, (1) beside (2) and (3) on the other
    half of each SIMD's waves)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    outs = []
    for i, arm in enumerate(({"ARL_CONV_EPW": "1", "ARL_FC_BIG": "0"}, {"ARL_CONV_EPW": "2", "ARL_FC_BIG": "0"},
                             {"ARL_CONV_EPW": "1", "ARL_FC_BIG": "1"}, {"ARL_WINDOW_C": "0"},
                             {"ARL_WINDOW_C": "0", "ARL_FUSE_RETURNS": "0"}, {"ARL_CB_WS": "0"})):
        f = str(tmp_path / f"arm_{i}.npz")
        env = dict(os.environ, **arm)
        subprocess.run([sys.executable, os.path.join(here, "conv_epw_worker.py"), f, str(n_envs)], env=env,
                       check=True, timeout=240)
        outs.append(np.load(f))
    assert float(np.abs(outs[0]["a2"]).max()) > 0
    for o in outs[1:]:
        for k in outs[0].files:
            assert np.array_equal(outs[0][k], o[k]), k


@pytest.mark.parametrize("arch,N", [("ff", 75), ("ff", 512), ("lstm", 80)])
def test_a2_mask_bits_match_a2(gpu, arch, N):
    """conv_fwd.hip's a2 > 0 bits (the FC backward's ReLU mask, 81 words per
    env-step, EPW 1 and 2) equal a2 > 0 in every sample slot of a window."""
    from asyncrl_amd import A3C, A3CFF, A3CLSTM, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(91)
    T, P = 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    Model = A3CLSTM if arch == "lstm" else A3CFF
    m = Model(4, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs")
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
    o.add_hook(GradientClipping(40))
    ag = A3C(m, o, T, 0.99)
    ag.run_window(dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu), P, first=True, env_groups=1)
    torch.cuda.synchronize()
    a2 = m.net.buffer("a2", torch.float32, (T + 1, N, 2592)).cpu().numpy()
    words = m.net.buffer("a2_mask", torch.int32, (T + 1, N, 81)).cpu().numpy().view(np.uint32)
    bits = (words[..., :, None] >> np.arange(32, dtype=np.uint32)) & 1
    # slots 0..T-1 (the bootstrap slot T feeds no backward: its mask and a1 are not stored)
    assert np.array_equal(bits.reshape(T + 1, N, 2592)[:T].astype(bool), a2[:T] > 0)
    assert float(np.abs(a2[T]).max()) > 0


def test_lstm_fc_ticket_big_tiles_identical(gpu, tmp_path):
    """512 LSTM envs (fc.hip's 64-row tiles): the FC forward's last-arriver
    ticket reduce (fc_fwd_big_kernel's tail, the default from 512-env
    launches) and the reduce in the gate kernel's staging sum the same partials in the same
    order, so hidden / cell states, gates, actions, gradients and parameters
    match bit for bit."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    outs = []
    for extra in ({"ARL_LSTM_XRED": "1"}, {"ARL_LSTM_XRED": "0"}):
        f = str(tmp_path / f"lstm512_{len(outs)}.npz")
        env = dict(os.environ, LSTM_WORKER_N="512", **extra)
        subprocess.run([sys.executable, os.path.join(here, "lstm_split_worker.py"), f], env=env, check=True,
                       timeout=240)
        outs.append(np.load(f))
    assert int((outs[0]["hbuf"] != 0).sum()) > 0
    for k in outs[0].files:
        assert np.array_equal(outs[0][k], outs[1][k]), k
