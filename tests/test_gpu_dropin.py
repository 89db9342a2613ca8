"""The reference-contract drop-in on the GPU: A3C.act(state, reward,
is_state_terminal) -> int | None on a one-env model, driven in the shape of
a3c_ale.py:100-126, against the REFERENCE's own a3c.py trajectories
(tests/golden/a3c_update_golden.npz, tests/a3c_golden.py); and the
A3CFF / A3CLSTM.pi_and_v(state, keep_same_state) / reset_state surface
(a3c_ale.py:38-40,55-66) against the oracle."""
import numpy as np
import pytest
import torch

import oracle as O
from a3c_golden import VARIANTS, load
from conftest import close_normscaled

RTOL = 1e-5   # fp32 device vs the reference run on the float64 stub


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _agent(v, gpu):
    from asyncrl_amd import A3C, A3CFF, A3CLSTM, GradientClipping, RMSpropAsync, dqn_phi
    Model = A3CFF if v.arch_name == "ff" else A3CLSTM
    model = Model(v.A, n_envs=1, t_max=v.T, seed=v.seed, init_seed=None, device=gpu)
    assert model.frames == "stacks"
    model.net.load_params(v.theta0())
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99)
    opt.setup(model)
    opt.add_hook(GradientClipping(v.clip))
    # dqn_phi variants: the uint8 stack ring; the *_phi variants' user phi: the f32 state ring
    phi = dqn_phi if v.phi is None else v.phi
    agent = A3C(model, opt, v.T, v.gamma, beta=v.beta, process_idx=0, phi=phi, pi_loss_coef=v.pi_loss_coef,
                v_loss_coef=v.v_loss_coef, keep_loss_scale_same=v.keep)
    assert model.frames == ("stacks" if v.phi is None else "states")
    return agent, model, opt


@pytest.mark.gpu
@pytest.mark.parametrize("name", VARIANTS)
def test_dropin_act_matches_reference_trajectory(gpu, name):
    v = load(name)
    agent, model, opt = _agent(v, gpu)
    net = model.net
    upd = list(v.update_calls)
    u = 0
    for k in range(v.n_calls):                       # a3c_ale.py:100-126
        opt.lr = float(v.lr[k])
        state = list(v.states[k])                    # ALE.state: 4 uint8 (84, 84) screens
        a = agent.act(state, float(v.rewards[k]), bool(v.terminals[k]))
        assert (-1 if a is None else a) == v.actions[k], (name, k, a)
        if a is not None:
            assert isinstance(a, int)
            o = net.step_outputs(agent.t - 1 - agent.t_start)
            assert rel(o["probs"].cpu().numpy()[0], v.probs[k]) < RTOL, (name, k)
            assert abs(float(o["entropy"][0]) - v.entropy[k]) <= RTOL * abs(v.entropy[k]), (name, k)
        if u < len(upd) and k == upd[u]:
            torch.cuda.synchronize()
            g = net.state_dict(net.grads)
            p = net.state_dict()
            for n in v.names:
                ok, err = close_normscaled(v.pick(n, g[n]), v.grad[n][u], RTOL)
                assert ok, (name, k, u, n, "grad", err)
                ok, err = close_normscaled(v.pick(n, p[n]), v.param[n][u], RTOL)
                assert ok, (name, k, u, n, "param", err)
            loss = net.buffer("loss", torch.float32, (1, 2)).cpu().numpy()[0]
            assert abs(loss[0] - v.loss[u, 0]) <= RTOL * max(abs(v.loss[u, 0]), 1e-3), (name, u, loss, v.loss[u])
            assert abs(loss[1] - v.loss[u, 1]) <= RTOL * max(abs(v.loss[u, 1]), 1e-3), (name, u, loss, v.loss[u])
            u += 1
    assert u == len(upd)


@pytest.mark.gpu
def test_dropin_phi_plugin(gpu):
    """The phi plugin (a3c.py:34,50,73): a user phi equal to dqn_phi's
    arithmetic runs on the f32 state ring and reproduces the reference's
    dqn_phi trajectory (actions, probabilities, first update's gradient); the
    default identity phi takes float32 states as they are; a phi whose output
    Chainer's Convolution2D would not take (uint8, float64) is refused."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    v = load("ff")

    def my_phi(screens):   # a user's phi, as in the reference (np.float32 / 255)
        return np.asarray(screens, dtype=np.float32) / np.float32(255.0)

    model = A3CFF(v.A, t_max=v.T, seed=v.seed, init_seed=None, device=gpu)
    model.net.load_params(v.theta0())
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(GradientClipping(v.clip))
    agent = A3C(model, opt, v.T, v.gamma, beta=v.beta, phi=my_phi)
    assert model.frames == "states" and model.net.states
    u0 = int(v.update_calls[0])
    for k in range(u0 + 1):
        opt.lr = float(v.lr[k])
        a = agent.act(list(v.states[k]), float(v.rewards[k]), bool(v.terminals[k]))
        assert (-1 if a is None else a) == v.actions[k], k
        if a is not None:
            o = model.net.step_outputs(agent.t - 1 - agent.t_start)
            assert rel(o["probs"].cpu().numpy()[0], v.probs[k]) < RTOL, k
    torch.cuda.synchronize()
    g = model.net.state_dict(model.net.grads)
    for n in v.names:
        ok, err = close_normscaled(v.pick(n, g[n]), v.grad[n][0], RTOL)
        assert ok, (n, err)
    # identity phi (the reference's default): float32 states go in as they are
    ident = A3C(A3CFF(v.A, t_max=v.T, device=gpu), RMSpropAsync(), v.T, v.gamma)
    assert ident.model.frames == "states"
    assert isinstance(ident.act(my_phi(list(v.states[0])), 0.0, False), int)
    with pytest.raises(ValueError):
        ident.act(np.asarray(v.states[1]), 0.0, False)                 # uint8: not a model input
    bad = A3C(A3CFF(v.A, t_max=v.T, device=gpu), RMSpropAsync(), v.T, v.gamma,
              phi=lambda s: my_phi(s).astype(np.float64))
    with pytest.raises(ValueError):
        bad.act(list(v.states[0]), 0.0, False)


@pytest.mark.gpu
def test_lstm_pi_and_v_state_semantics(gpu):
    """A3CLSTM.pi_and_v(state, keep_same_state) and reset_state
    (a3c_ale.py:55-66) against the oracle's L.LSTM restatement: the state
    advances per call, keep_same_state leaves it, reset_state clears it."""
    from asyncrl_amd import A3CLSTM
    rng = np.random.default_rng(31)
    A, n = 6, 3
    model = A3CLSTM(A, n_envs=n, t_max=5, init_seed=8, device=gpu)
    params = model.net.state_dict()
    xs = O.PHI_LUT[rng.integers(0, 256, (7, n, 4, 84, 84), dtype=np.uint8)]
    h = np.zeros((n, 256), np.float32)
    c = np.zeros((n, 256), np.float32)
    has = np.zeros(n, bool)
    script = [False, False, True, False, "reset", False, True]
    for k, op in enumerate(script):
        if op == "reset":
            model.reset_state()
            has[:] = False
            continue
        keep = bool(op)
        pout, vv = model.pi_and_v(torch.from_numpy(xs[k]).to(gpu), keep_same_state=keep)
        _, _, hfc = O.nips_head(params, O.ARCH_LSTM, xs[k])
        _, c2, h2 = O.lstm_cell(params, O.ARCH_LSTM, hfc, h, c, has)
        logits = O.linear(h2, params["2/0/W"], params["2/0/b"])
        vo = O.linear(h2, params["3/0/W"], params["3/0/b"])[:, 0]
        ok, err = close_normscaled(pout.logits.cpu().numpy(), logits, RTOL)
        assert ok, (k, err)
        ok, err = close_normscaled(vv.cpu().numpy(), vo, RTOL)
        assert ok, (k, err)
        if not keep:
            h, c, has = h2, c2, np.ones(n, bool)


@pytest.mark.gpu
def test_pi_and_v_draws_afresh_each_call(gpu):
    """Repeated sampling pi_and_v calls on the same state are independent
    draws from the policy (not one fixed quantile); the returned
    tensors are copies that later calls do not overwrite."""
    from scipy.stats import chisquare
    from asyncrl_amd import A3CFF
    rng = np.random.default_rng(5)
    model = A3CFF(4, n_envs=1, t_max=5, init_seed=2, device=gpu)
    x = torch.from_numpy(O.PHI_LUT[rng.integers(0, 256, (1, 4, 84, 84), dtype=np.uint8)]).to(gpu)
    first, _ = model.pi_and_v(x)
    a0 = first.action_indices.clone()
    draws = []
    for _ in range(3000):
        pout, _ = model.pi_and_v(x)
        draws.append(pout.action_indices)
    assert torch.equal(first.action_indices, a0)
    acts = torch.cat(draws).cpu().numpy()
    p = first.probs.cpu().numpy()[0].astype(np.float64)
    counts = np.bincount(acts, minlength=4)
    assert chisquare(counts, p / p.sum() * len(acts)).pvalue > 1e-4, (counts, p)
