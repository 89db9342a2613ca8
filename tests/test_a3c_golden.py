"""The oracle's A3C update against the reference's own a3c.py trajectories
(tests/golden/a3c_update_golden.npz, see tests/a3c_golden.py): the oracle's
one-env agent (oracle.A3CAgent, a restatement of a3c.py:67-167 with
GradientClipping + RMSpropAsync) replays every act call of each variant and
must reproduce the reference's actions exactly and its policy outputs,
returns, losses, gradient norms, gradients and post-update parameters
within the fp32 tolerance below.  Pins rows a13-a19 (and the pi_loss_coef /
v_loss_coef / keep_loss_scale_same options) to the reference's code."""
import numpy as np
import pytest

import oracle as O
from a3c_golden import VARIANTS, load
from conftest import close_normscaled

RTOL = 1e-5   # fp32 vs the stub's float64 truth, |a - b| <= RTOL * max(|b|, ||b||_inf)


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def test_fixture_covers_the_update_paths():
    """Each variant holds full-window (bootstrapped) and terminal-truncated
    updates of several lengths; the *_opts variants clip every update."""
    for name in VARIANTS:
        v = load(name)
        L = v.window_lengths()
        term = [bool(v.terminals[k]) for k in v.update_calls]
        assert any(not t for t in term) and any(term), name
        assert any(ln < v.T for ln, t in zip(L, term) if t), name
        assert len(set(L)) >= 3, (name, L)
        if v.clip < 1:
            assert (v.grad_norm > v.clip).all(), name


@pytest.mark.parametrize("name", VARIANTS)
def test_oracle_agent_replays_reference(name):
    v = load(name)
    ag = O.A3CAgent(v.theta0(), v.arch, v.A, v.T, v.gamma, v.beta, v.pi_loss_coef, v.v_loss_coef, v.keep,
                    v.clip, v.seed, phi=v.phi)
    for k in range(v.n_calls):
        a = ag.act(v.states[k], v.rewards[k], bool(v.terminals[k]), float(v.lr[k]))
        assert (-1 if a is None else a) == v.actions[k], (name, k)
        if a is not None:
            c = ag.calls[-1]
            assert rel(c["probs"], v.probs[k]) < RTOL, (name, k)
            assert abs(c["entropy"] - v.entropy[k]) <= RTOL * abs(v.entropy[k]), (name, k)
    assert [u["call"] for u in ag.updates] == v.update_calls.tolist()
    for u, up in enumerate(ag.updates):
        L = up["L"]
        assert rel(up["R"], v.R[u, :L]) < RTOL, (name, u)
        assert rel(up["v"], v.v[u, :L]) < RTOL, (name, u)
        assert abs(up["pi_loss"] - v.loss[u, 0]) <= RTOL * max(abs(v.loss[u, 0]), 1e-3), (name, u)
        assert abs(up["v_loss"] - v.loss[u, 1]) <= RTOL * max(abs(v.loss[u, 1]), 1e-3), (name, u)
        assert abs(up["norm"] - v.grad_norm[u]) <= RTOL * v.grad_norm[u], (name, u)
        for n in v.names:
            ok, err = close_normscaled(v.pick(n, up["grads"][n]), v.grad[n][u], RTOL)
            assert ok, (name, u, n, err)
            ok, err = close_normscaled(v.pick(n, up["params"][n]), v.param[n][u], RTOL)
            assert ok, (name, u, n, "param", err)
