"""Derived device state stays coherent with the parameters (ABI 4 parameter
generations).  The FC forward reads its weight as bf16 split planes derived
from the f32 params; every write of the params that the library does not make
itself must bump the net's parameter generation, or the next forward runs on
the old W.  Each test writes the params one way, then checks the next forward
against the oracle on the new params (1e-5 norm-scaled); the stale
arm (the bump skipped) must fail that same check.  Reference writers:
copy_param.py:1-6 (shared -> local params), a3c.py:139-143 (update, sync),
serializers.load_hdf5 (demo_a3c_ale.py:61)."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import close_normscaled
from sim import make_pools

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def dev(x, gpu):
    return torch.from_numpy(np.ascontiguousarray(x)).to(gpu)


def _forward_ok(model, stacks, gpu):
    """pi_and_v on dqn_phi(stacks) against the oracle on the net's current
    params: (ok, err) of the logits and values."""
    from asyncrl_amd import dqn_phi
    pout, v = model.pi_and_v(dqn_phi(dev(stacks, gpu)))
    lo, vo, _ = O.pi_and_v_ff(model.net.state_dict(), O.PHI_LUT[stacks])
    ok1, e1 = close_normscaled(pout.logits.cpu().numpy(), lo, RTOL)
    ok2, e2 = close_normscaled(v.cpu().numpy(), vo, RTOL)
    return ok1 and ok2, max(e1, e2)


def _model(n=24, seed=3):
    from asyncrl_amd import A3CFF
    return A3CFF(4, n_envs=n, t_max=5, init_seed=seed)


def _stacks(n=24):
    return np.random.default_rng(31).integers(0, 256, (n, 4, 84, 84), dtype=np.uint8)


@pytest.mark.parametrize("stale", [False, True])
def test_update_arrays_on_net_params_rebuilds_planes(gpu, monkeypatch, stale):
    """RMSpropAsync.update_arrays (the drop-in for update_one_cpu on one
    array) applied to a net's own params: the kernel writes them behind
    torch's back, so update_arrays bumps the generation of every net whose
    params it aliases.  stale=True skips that bump: the forward must then
    disagree with the oracle (the test can fail)."""
    from asyncrl_amd import RMSpropAsync
    from asyncrl_amd import rmsprop_async
    model, stacks = _model(), _stacks()
    net = model.net
    assert _forward_ok(model, stacks, gpu)[0]           # planes built from the init params
    if stale:
        monkeypatch.setattr(rmsprop_async, "nets_aliasing", lambda t: [])
    g = torch.from_numpy(np.random.default_rng(5).normal(0, 1, net.param_floats).astype(np.float32)).to(gpu)
    ms = torch.zeros_like(net.params)
    RMSpropAsync(lr=0.05, alpha=0.99, eps=0.1).update_arrays(net.params, ms, g)
    torch.cuda.synchronize()
    pg, plg = net.param_generation()
    assert (pg != plg) != stale                          # the bump happened (or, in the stale arm, did not)
    ok, err = _forward_ok(model, stacks, gpu)
    assert ok != stale, err


def test_inplace_writes_through_views_and_setter_rebuild_planes(gpu):
    """Writes through the params tensor or a view of it (torch's version
    counter) and `net.params = x` (copy into the bound memory + bump) are
    both seen before the next forward."""
    model, stacks = _model(), _stacks()
    net = model.net
    assert _forward_ok(model, stacks, gpu)[0]
    net.param("0/2/W").mul_(-1.5)                        # the FC weight, in place through a view
    assert _forward_ok(model, stacks, gpu)[0]
    fresh = _model(seed=8).net.params.clone()
    net.params = fresh
    assert torch.equal(net.params, fresh)
    assert _forward_ok(model, stacks, gpu)[0]


def test_load_params_after_windows_matches_fresh_net(gpu):
    """Run windows (the in-window update keeps the planes current), load new
    weights, forward: equal to a fresh net built with those weights."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(41)
    N, T, P = 24, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    model = A3CFF(4, n_envs=N, t_max=T, init_seed=1, frames="pairs")
    o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(model)
    o.add_hook(GradientClipping(40))
    ag = A3C(model, o, T, 0.99)
    for w in range(2):
        ag.run_window(dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu), P, first=(w == 0))
    new = _model(n=N, seed=9)
    model.net.load_params(new.net.state_dict())
    stacks = _stacks(N)
    assert _forward_ok(model, stacks, gpu)[0]
    from asyncrl_amd import dqn_phi
    x = dqn_phi(dev(stacks, gpu))
    a, b = model.pi_and_v(x)[0].logits, new.pi_and_v(x)[0].logits
    assert torch.equal(a, b)


def test_graph_replay_after_load_needs_prepare(gpu):
    """A captured window holds no plane rebuild: after load_params, prepare()
    on the replay stream makes the replay's forward use the loaded weights --
    bit-identical to an eager window on a net that loaded them first."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(43)
    N, T, P = 16, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    w_new = _model(n=N, seed=12).net.state_dict()

    def mk():
        m = A3CFF(4, n_envs=N, t_max=T, seed=3, init_seed=4, frames="pairs")
        o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
        o.add_hook(GradientClipping(40))
        return A3C(m, o, T, 0.99)

    a, b = mk(), mk()
    a.run_window(dp, dr, dd, P, first=True)
    a.net.load_params(w_new)
    a.run_window(dp, dr, dd, P)
    b.run_window(dp, dr, dd, P, first=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        b.run_window(dp, dr, dd, P)
    b.net.load_params(w_new)           # written after the capture
    with torch.cuda.stream(s):
        b.net.prepare(s)
        g.replay()
    torch.cuda.synchronize()
    assert b.net.param_generation()[0] == b.net.param_generation()[1]
    assert torch.equal(a.net.params, b.net.params)


def test_env_groups_first_window_after_params_changed(gpu):
    """params_changed() and then a first=True window with two env
    groups -- the planes are rebuilt on the main stream before the chains
    fork (A3C.run_window -> DeviceNet.prepare), so the result equals one
    group bit for bit; and an env-range act on stale planes is refused
    (ARL_ESTATE) instead of racing."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    rng = np.random.default_rng(47)
    N, T, P = 256, 5, 7
    pairs, rewards, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    dp, dr, dd = dev(pairs, gpu), dev(rewards, gpu), dev(dones, gpu)
    outs = []
    for G in (1, 2):
        m = A3CFF(4, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs")
        o = RMSpropAsync(lr=7e-4, eps=0.1, alpha=0.99).setup(m)
        o.add_hook(GradientClipping(40))
        ag = A3C(m, o, T, 0.99)
        m.net.params_changed()
        if G == 2:
            m.net.observe(0, dp, dr, dd, P, force_reset=True, envs=(0, 128))
            with pytest.raises(RuntimeError, match="arl_net_prepare"):
                m.net.act(0, envs=(0, 128))
        ag.run_window(dp, dr, dd, P, first=True, env_groups=G)
        torch.cuda.synchronize()
        outs.append((m.net.params.clone(), m.net.grads.clone(),
                     m.net.buffer("actions", torch.int32, (T + 1, N)).clone()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_dropped_fused_window_does_not_skip_returns(gpu):
    """a fused bootstrap act (returns run inside the policy
    launch) whose learn never follows must not make a later window's learn
    skip its own returns.  Window 1 is issued with the fusion on and dropped;
    window 2 (other rewards) is issued step by step without fusion and
    learned: its gradient equals a net that only ran window 2."""
    from asyncrl_amd import A3CFF
    rng = np.random.default_rng(53)
    N, T, P = 32, 5, 6
    pairs, r1, dones = make_pools(rng, P, N, "uniform", p_done=0.1)
    r2 = np.where(r1 == 0, 1.0, 0.0).astype(np.float32)
    dp, dd = dev(pairs, gpu), dev(dones, gpu)

    def chain(net, rw):
        for t in range(T + 1):
            net.observe(t, dp, dev(rw, gpu), dd, P, force_reset=(t == 0))
            net.act(t, mode=1 if t < T else 0)

    grads = []
    for drop in (True, False):
        m = A3CFF(4, n_envs=N, t_max=T, seed=5, init_seed=6, frames="pairs")
        net = m.net
        net.reset()
        if drop:
            net.set_returns_fusion(True)
            chain(net, r1)
            net.set_returns_fusion(False)
        chain(net, r2)
        net.grads.zero_()
        net.learn()
        torch.cuda.synchronize()
        grads.append(net.grads.clone())
    assert float(grads[0].abs().max()) > 0
    assert torch.equal(grads[0], grads[1])
