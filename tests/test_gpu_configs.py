"""Parity at BASELINE.json's full per-GPU config sizes (the bench workloads),
against the CPU oracle -- everything except C4's RCCL exchange, which needs
more than one GPU:

  C3  A3C LSTM, 1024 envs, A = 6, the default two env groups, two windows
  C4  the per-GPU leg of the 8-GPU config: A3C FF, 512 envs, two env groups
  C2  A3C FF, 256 envs, two windows
(each on uniform frames and on SURVEY 8(d)'s shaped frames: palette blocks on
black, all-255 envs and uniform envs in one batch)
  C5  phi_stack over 16,384 frame pairs (a 3.3 GB input whose byte offsets
      pass 2^31)

The oracle runs over env chunks (envs are independent until the learner
sums their gradients) and sums the chunk gradients in float64.
Tolerance: forward outputs |gpu - oracle| <= 1e-5 * max(|oracle|,
||oracle||_inf) per tensor; gradients componentwise, |gpu -
oracle| <= 1e-5 * (L2 norm of the element's summands) (conftest.close_grad)."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import close_normscaled, grads_match
from sim import OracleEnvView, make_pools, oracle_window_chunks as _oracle_window

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def dev(x, gpu):
    return torch.from_numpy(np.ascontiguousarray(x)).to(gpu)


def _run_config(gpu, arch, N, A, windows=2, seed=0, kind="uniform", env_groups=None):
    from asyncrl_amd import A3C, A3CFF, A3CLSTM, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(seed)
    T, P = 5, 6          # pool of 6 steps, reused cyclically by the second window
    pairs, rewards, dones = make_pools(rng, P, N, kind, p_done=0.1)
    Model = A3CLSTM if arch == O.ARCH_LSTM else A3CFF
    model = Model(A, n_envs=N, t_max=T, seed=77, init_seed=seed + 1, frames="pairs", device=gpu)
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(GradientClipping(40))
    agent = A3C(model, opt, T, 0.99)
    net = model.net
    groups = net.env_groups(net.default_env_groups() if env_groups is None else env_groups)
    view = OracleEnvView(pairs, dones)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    st = O.LSTMState(h=np.zeros((N, 256), np.float32), c=np.zeros((N, 256), np.float32), has=np.zeros(N, bool))
    prev_done = np.ones(N, np.uint8)
    for w in range(windows):
        k0 = w * T
        params = net.state_dict()
        agent.run_window(dp, dr, dd, P, first=(w == 0), split_update=True, env_groups=len(groups))
        torch.cuda.synchronize()
        states, boot = view.states_f32(k0, T)
        r, d = view.window_rd(rewards, k0, T)
        acts = net.buffer("actions", torch.int32, (T + 1, N))[:T].cpu().numpy()
        dprev = np.concatenate([prev_done[None], d[:-1]], 0)
        acts_dev = (net.buffer("a1", torch.float32, (T + 1, N, 16, 20, 20))[:T].cpu().numpy(),
                    net.buffer("a2", torch.float32, (T + 1, N, 32, 9, 9))[:T].cpu().numpy(),
                    net.buffer("hfc", torch.float32, (T + 1, N, 256))[:T].cpu().numpy())
        g, aux = _oracle_window(arch, params, states, acts, r, d, boot, st, dprev, acts_dev)
        logits = net.buffer("logits", torch.float32, (T + 1, N, A))[:T].cpu().numpy()
        v = net.buffer("v", torch.float32, (T + 1, N)).cpu().numpy()
        for name, got, want in (("logits", logits, aux["logits"]), ("v", v[:T], aux["v"]),
                                ("vboot", v[T], aux["vboot"]),
                                ("dlogits", net.buffer("dlogits", torch.float32, (T, N, A)).cpu().numpy(),
                                 aux["dlogits"]),
                                ("dv", net.buffer("dv", torch.float32, (T, N)).cpu().numpy(), aux["dv"])):
            ok, err = close_normscaled(got, want, RTOL)
            assert ok, (w, name, err)
        probs = net.buffer("probs", torch.float32, (T + 1, N, A)).cpu().numpy()
        for t in range(T):
            u = O.sample_uniforms(77, np.arange(N, dtype=np.uint64), k0 + t)
            assert (O.sample_from_uniform(probs[t], u) == acts[t]).all(), (w, t)
        grads_match(net.state_dict(net.grads), g, aux["grad_mag"], RTOL)
        agent.finish_window()
        if arch == O.ARCH_LSTM:
            st = O.LSTMState(h=aux["h_last"], c=aux["c_last"], has=np.ones(N, bool))
        prev_done = d[-1]
    return groups


def test_c3_lstm_1024_envs_two_groups(gpu):
    groups = _run_config(gpu, O.ARCH_LSTM, 1024, 6, seed=3)
    assert len(groups) == 2


def test_c3_lstm_1024_envs_shaped_frames(gpu):
    """C3 on SURVEY 8(d)'s shaped frames: sparse palette blocks on black
    (conv pre-activations tie at zero: the tie-aware ReLU masks), all-255 envs
    and uniform envs mixed in one batch."""
    _run_config(gpu, O.ARCH_LSTM, 1024, 6, seed=13, kind="shaped")


@pytest.mark.parametrize("env_groups", [None, 2])
def test_c4_leg_ff_512_envs(gpu, env_groups):
    """The C4 per-GPU leg: the default one chain of 512 envs (two envs a conv
    workgroup, 64-row FC tiles) and two chains of 256 (two envs a conv
    workgroup, 32-row FC tiles)."""
    groups = _run_config(gpu, O.ARCH_FF, 512, 4, seed=4, env_groups=env_groups)
    assert len(groups) == (1 if env_groups is None else 2)


def test_c2_ff_256_envs(gpu):
    _run_config(gpu, O.ARCH_FF, 256, 4, seed=2)


def test_c2_ff_256_envs_shaped_frames(gpu):
    _run_config(gpu, O.ARCH_FF, 256, 4, seed=12, kind="shaped")


def test_c4_leg_ff_512_envs_shaped_frames(gpu):
    _run_config(gpu, O.ARCH_FF, 512, 4, seed=14, kind="shaped")


def test_c5_phi_stack_16384_pairs(gpu):
    """C5: one materialised phi_stack over 16,384 pairs (3.3 GB in).  Envs
    past byte offset 2^31 (env >= 10,653) and both ends are checked
    bit-exact against the oracle; every env is checked by two
    size-independent properties: planes 0-2 are the previous stack shifted
    (zeros after a reset) and plane 3 equals the single-screen kernel
    (arl_current_screen) on the same pair."""
    from asyncrl_amd import current_screen, phi_stack
    n = 16384
    g = torch.Generator(device=gpu).manual_seed(5)
    pairs = torch.randint(0, 256, (n, 2, 210, 160, 3), dtype=torch.uint8, device=gpu, generator=g)
    prev = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=gpu, generator=g)
    reset = (torch.rand(n, device=gpu, generator=g) < 0.3).to(torch.uint8)
    out = phi_stack(pairs, prev, reset)
    torch.cuda.synchronize()
    shifted = torch.where(reset.bool()[:, None, None, None], torch.zeros_like(prev[:, 1:]), prev[:, 1:])
    assert torch.equal(out[:, :3], shifted)
    for e0 in range(0, n, 4096):
        scr = current_screen(pairs[e0:e0 + 4096, 0].contiguous(), pairs[e0:e0 + 4096, 1].contiguous())
        assert torch.equal(out[e0:e0 + 4096, 3], scr), e0
    first_high = -(-(1 << 31) // (2 * 210 * 160 * 3))
    check = sorted({0, 1, first_high - 1, first_high, first_high + 1, n - 2, n - 1} |
                   set(np.random.default_rng(6).integers(first_high, n, 8).tolist()))
    idx = torch.tensor(check, device=gpu)
    hp, hprev = pairs[idx].cpu().numpy(), prev[idx].cpu().numpy()
    ho, hr = out[idx].cpu().numpy(), reset[idx].cpu().numpy()
    for j, e in enumerate(check):
        scr = O.current_screen(hp[j, 0], hp[j, 1])
        assert (ho[j] == O.stack_push(hprev[j], scr, bool(hr[j]))).all(), e
