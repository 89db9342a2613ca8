"""Batched evaluation episodes (a3c_ale.py:73-89,
demo_a3c_ale.py:15-30): N envs of a VecALE play greedy episodes through the
model's device workspace.  Checked against a serial replay on the CPU: the
same emulators (FakeALE, seeded no-op counts), life loss not terminal, the
oracle's frame stacks and pi_and_v, and at every step the device's action
must be an argmax of the oracle's policy (tie-aware: within 1e-5 of the
maximum probability); the replay then follows the device's action, so the
episode scores must match exactly."""
import statistics

import numpy as np
import pytest
import torch

from fake_ale import FakeALEActions

import oracle as O
from asyncrl_amd.envs import ALEFramePairs, VecALE


def _serial_replay(params, n, seed, nullops, actions):
    """The reference's eval loop per env over the device's action trace:
    returns per-env lists of episode scores and the count of steps checked."""
    envs = [ALEFramePairs(FakeALEActions(), nullop_rng=np.random.RandomState(seed + i),
                          max_start_nullops=nullops) for i in range(n)]
    for e in envs:
        e.treat_life_lost_as_terminal = False   # ale.ALE(rom, treat_life_lost_as_terminal=False)
        e.ale.reset_game()                      # a fresh game per eval run (a3c_ale.py:75-76)
        e.initialize()
    stacks = [O.stack_push(None, O.current_screen(e.pair[0], e.pair[1]), True) for e in envs]
    scores = [[] for _ in range(n)]
    acc = [0.0] * n
    for k, acts in enumerate(actions):
        x = np.stack([O.dqn_phi(list(s)) for s in stacks])
        logits, _, _ = O.pi_and_v_ff(params, x)
        probs = O.softmax(logits.astype(np.float64))
        for i, e in enumerate(envs):
            a = int(acts[i])
            assert probs[i, a] >= probs[i].max() - 1e-5, (k, i, probs[i], a)
            pair, r, done = e.step(a)
            acc[i] += r
            if done:
                scores[i].append(acc[i])
                acc[i] = 0.0
            stacks[i] = O.stack_push(stacks[i], O.current_screen(pair[0], pair[1]), done)
    return scores


@pytest.mark.gpu
@pytest.mark.parametrize("n_envs,n_runs", [(3, 5), (4, 4)])
def test_eval_greedy_matches_serial_replay(gpu, n_envs, n_runs):
    from asyncrl_amd import A3CFF, eval_performance, run_episodes
    seed, nullops = 5, 4
    vec = VecALE([FakeALEActions() for _ in range(n_envs)], device=gpu, seed=seed, max_start_nullops=nullops)
    model = A3CFF(vec.number_of_actions, n_envs=n_envs, t_max=5, seed=3, init_seed=7, frames="pairs")
    scores, trace = run_episodes(model, vec, n_runs, deterministic=True, max_steps=500)
    torch.cuda.synchronize()
    params = model.net.state_dict()
    per_env = _serial_replay(params, n_envs, seed, nullops, trace["actions"])
    want = np.array([per_env[k % n_envs][k // n_envs] for k in range(n_runs)])
    assert (scores == want).all(), (scores, want)
    # life loss is not terminal: FakeALE loses a life at frame 22 and ends at 41,
    # so every episode spans a life loss
    assert all(e.treat_life_lost_as_terminal for e in vec.envs)   # restored afterwards
    # the (mean, median, stdev) summary of a3c_ale.py:85-88 over the same runs
    vec2 = VecALE([FakeALEActions() for _ in range(n_envs)], device=gpu, seed=seed, max_start_nullops=nullops)
    model.net.reset()
    got = eval_performance(model, vec2, n_runs, deterministic=True, max_steps=500)
    s = [float(x) for x in want]
    assert got == (statistics.mean(s), statistics.median(s), statistics.stdev(s))
    vec.close()
    vec2.close()


@pytest.mark.gpu
def test_eval_sampled_and_lstm_run(gpu):
    """Sampling mode (the training script's eval) and the LSTM model: the
    episodes finish, every action is legal, scores are the per-episode sums
    of the rewards the envs returned."""
    from asyncrl_amd import A3CFF, A3CLSTM, run_episodes
    for cls, det in ((A3CFF, False), (A3CLSTM, True), (A3CLSTM, False)):
        vec = VecALE([FakeALEActions() for _ in range(3)], device=gpu, seed=9, max_start_nullops=2)
        model = cls(vec.number_of_actions, n_envs=3, t_max=4, seed=1, init_seed=2, frames="pairs")
        scores, trace = run_episodes(model, vec, 6, deterministic=det, max_steps=500)
        a, d = trace["actions"], trace["dones"]
        assert a.min() >= 0 and a.max() < vec.number_of_actions
        assert d.sum(0).min() >= 2 and np.isfinite(scores).all() and (scores >= 0).all()
        vec.close()


def test_eval_rejects_bad_setups():
    """Host-side checks before any device work."""
    from asyncrl_amd.evaluation import eval_performance, run_episodes

    class M:
        class net:
            n_envs, t_max = 2, 5
        frames = "pairs"

    vec = VecALE([FakeALEActions() for _ in range(3)], device="cpu", seed=0, max_start_nullops=0)
    with pytest.raises(ValueError):
        run_episodes(M, vec, 4)                 # 3 envs vs a 2-env workspace
    with pytest.raises(ValueError):
        eval_performance(M, vec, 1)             # stdev needs two runs (a3c_ale.py:74)
    vec.close()
