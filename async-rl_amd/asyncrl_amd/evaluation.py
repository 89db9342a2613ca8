"""Batched evaluation episodes.

The reference evaluates one episode at a time on the CPU: a fresh
`ale.ALE(rom, treat_life_lost_as_terminal=False)` per run, dqn_phi of the
frame stack, one `pi_and_v` per step, the sampled action (a3c_ale.py:73-89)
or, in the demo's deterministic mode, `most_probable_actions`
(demo_a3c_ale.py:15-30), the raw game reward summed until game over, then
mean / median / stdev over the runs.

Here the N envs of a `VecALE` run their episodes in lockstep through the
model's own device workspace -- the same phi ring, forward and policy
kernels the training window uses (`arl_observe` + `arl_act_mode`: mode 2 =
first argmax, mode 1 = a Philox draw) -- so one batched forward serves N
episodes per step.  An env that finishes an episode starts its next one at
once (VecALE's batched convention: the done flag of an observation resets
its frame stack and LSTM state on the device).  Episode k of env i is run
number k * N + i; the first `n_runs` run numbers are the scores returned, so
the result does not depend on which env finishes first.

Life loss is not terminal here (the reference's eval ALE), whatever the
envs were built with: `eval_performance` switches it off for the duration,
and every env's game restarts at the start of the evaluation.  The envs are
left partway through episodes when it returns.
The run uses (and overwrites) the model's lockstep workspace -- frame ring,
step counter, LSTM state -- so evaluate on a model of its own (copy the
trained parameters in: `eval_model.net.copy_params_from(model.net)`), and
on a VecALE of its own: every env's game is restarted and left mid-episode,
so a training learner stepping the same envs would carry its frame ring,
LSTM state and n-step bootstrap across an unrelated game without a terminal
(the reference builds a fresh ALE per evaluation run, a3c_ale.py:75-76).
Host-side driver code; the per-step work is the device forward.
"""
from __future__ import annotations

import statistics

import numpy as np

MODE_SAMPLE, MODE_GREEDY = 1, 2


def run_episodes(model, vec_env, n_runs: int, deterministic: bool = False, max_steps: int | None = None,
                 stream=None):
    """Run `n_runs` evaluation episodes over `vec_env` (a VecALE with exactly
    model.net.n_envs envs, not the training learner's: its games restart)
    with the model's lockstep workspace.  Returns
    (scores, trace): scores[k] is the raw reward sum of run k (run k = env
    k % N's (k // N)-th episode); trace holds per-step host copies of the
    actions and done flags, (steps, N) each, for checking."""
    net = model.net
    N, T = net.n_envs, net.t_max
    if vec_env.n != N:
        raise ValueError(f"eval: VecALE has {vec_env.n} envs, the model's workspace {N}")
    if n_runs < 1:
        raise ValueError("eval: n_runs must be >= 1")
    if getattr(model, "frames", "pairs") != "pairs":
        raise ValueError("eval: the model must take frame pairs (frames='pairs')")
    mode = MODE_GREEDY if deterministic else MODE_SAMPLE
    need = [len(range(i, n_runs, N)) for i in range(N)]     # episodes env i must finish
    saved = [e.treat_life_lost_as_terminal for e in vec_env.envs]
    scores = np.zeros(n_runs, np.float64)
    trace_a, trace_d = [], []
    try:
        for e in vec_env.envs:
            # a fresh game per env, as the reference builds a fresh ALE per eval run
            # (a3c_ale.py:75-76): an env left mid-game by training starts over
            e.treat_life_lost_as_terminal = False
            e.ale.reset_game()
            e.initialize()
        pairs, r, d = vec_env.reset(stream)
        done_eps = [0] * N
        acc = np.zeros(N, np.float64)
        # slots 0..T-1 of a window, then advance: slot 0 of the next window is
        # the ring position observe(T) filled, its reset flags and LSTM carry
        # (hbuf[T] = the state after slot T-1) moved there, exactly as the
        # training window continues (net.hip advance_kernel)
        net.observe(0, pairs, r, d, 1, force_reset=True, stream=stream)
        t, steps = 0, 0
        while any(done_eps[i] < need[i] for i in range(N)):
            if max_steps is not None and steps >= max_steps:
                raise RuntimeError(f"eval: {max_steps} steps without finishing {n_runs} runs")
            net.act(t, mode=mode, stream=stream)
            acts = net.step_outputs(t)["actions"].clone()
            pairs, r, d = vec_env.step(acts, stream)
            hr, hd = r.cpu().numpy(), d.cpu().numpy()
            trace_a.append(acts.cpu().numpy())
            trace_d.append(hd.copy())
            for i in range(N):
                if done_eps[i] >= need[i]:
                    continue                     # this env's runs are complete: its steps are ignored
                acc[i] += float(hr[i])
                if hd[i]:
                    scores[done_eps[i] * N + i] = acc[i]
                    done_eps[i] += 1
                    acc[i] = 0.0
            steps += 1
            net.observe(t + 1, pairs, r, d, 1, stream=stream)
            t += 1
            if t == T:
                net.advance(stream)
                t = 0
    finally:
        for e, s in zip(vec_env.envs, saved):
            e.treat_life_lost_as_terminal = s
    return scores, {"actions": np.array(trace_a), "dones": np.array(trace_d)}


def eval_performance(model, vec_env, n_runs: int, deterministic: bool = False, max_steps: int | None = None,
                     stream=None):
    """a3c_ale.py:73-89 batched: (mean, median, stdev) of `n_runs` episode
    scores.  By default the action is sampled from the policy, as the
    training script's eval does (pout.action_indices); deterministic=True
    plays most_probable_actions (demo_a3c_ale.py:15-30)."""
    if n_runs < 2:
        raise ValueError("Computing stdev requires at least two runs")   # a3c_ale.py:74
    scores, _ = run_episodes(model, vec_env, n_runs, deterministic, max_steps, stream)
    s = [float(x) for x in scores]
    return statistics.mean(s), statistics.median(s), statistics.stdev(s)
