"""CPU baseline: the oracle's restatement of ONE reference actor-learner
process (a3c_ale.py:92-171 train_loop -> a3c.py:67-167 act), batch 1,
single-threaded (OMP_NUM_THREADS=1 as at a3c_ale.py:186), timed on the host.

TEST / BASELINE INFRASTRUCTURE ONLY (imported by bench.py's cpu_baseline leg).
run() is leg (i), one process on one core; run_parallel() leg (ii), P
processes in the reference's style.
Per env-step: ale.py:59-89 current_screen + deque push, dqn_phi, NIPS-head
forward + heads (batch 1), softmax / log-softmax / entropy, one draw; every
t_max steps: bootstrap forward, n-step returns, backward over the window,
GradientClipping(40), RMSpropAsync over all 677,429 parameters -- the same
work the reference does per step minus the emulator.
"""
from __future__ import annotations

import time

import numpy as np

import oracle as O
O.EXACT_SUMS = False   # time the f32 arithmetic Chainer does


def run(seconds: float = 10.0, t_max: int = 5, n_actions: int = 4, seed: int = 0, pool: int = 16):
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(1)
    except Exception:  # pragma: no cover
        limiter = None
    rng = np.random.default_rng(seed)
    params = O.init_like_torch(O.ARCH_FF, n_actions, rng)
    ms = {k: np.zeros_like(v) for k, v in params.items()}
    frames = rng.integers(0, 256, (pool, 2, 210, 160, 3), dtype=np.uint8)
    rewards = rng.choice(np.array([-1.0, 0.0, 1.0], np.float32), pool, p=[0.025, 0.95, 0.025])
    dones = (rng.random(pool) < 1 / 500).astype(np.uint8)
    names = list(params)
    stack = O.stack_push(None, O.current_screen(frames[0, 0], frames[0, 1]), True)
    steps = 0
    buf = []
    t0 = time.perf_counter()
    deadline = t0 + seconds
    while True:
        k = steps % pool
        x = O.PHI_LUT[stack][None]
        logits, v, acts = O.pi_and_v_ff(params, x)
        p = O.softmax(logits)
        lp = O.log_softmax(logits)
        u = O.sample_uniforms(seed, np.zeros(1, np.uint64), steps)
        a = O.sample_from_uniform(p, u)
        buf.append((x, acts, p, lp, v, a))
        # env transition: next observation (phi), reward, terminal
        j = (k + 1) % pool
        scr = O.current_screen(frames[j, 0], frames[j, 1])
        stack = O.stack_push(stack, scr, bool(dones[j]))
        steps += 1
        if steps % t_max == 0:
            xb = O.PHI_LUT[stack][None]
            _, vb, _ = O.pi_and_v_ff(params, xb)
            T = len(buf)
            r = np.array([[rewards[(steps - T + i + 1) % pool]] for i in range(T)], np.float32)
            d = np.array([[dones[(steps - T + i + 1) % pool]] for i in range(T)], np.uint8)
            probs = np.stack([b[2] for b in buf])
            logp = np.stack([b[3] for b in buf])
            vals = np.stack([b[4] for b in buf])
            act = np.stack([b[5] for b in buf])
            _, _, dl, dv, _, _ = O.returns_and_lossgrad(r, d, vals, vb, probs, logp, act)
            xs = np.concatenate([b[0] for b in buf])
            a1 = np.concatenate([b[1][0] for b in buf])
            a2 = np.concatenate([b[1][1] for b in buf])
            hh = np.concatenate([b[1][2] for b in buf])
            g = O.ff_backward(params, xs, (a1, a2, hh), dl.reshape(T, -1), dv.reshape(T))
            gl, _ = O.clip_grads([g[n] for n in names], 40.0)
            for n, gn in zip(names, gl):
                params[n], ms[n] = O.rmsprop_update(params[n], ms[n], gn, 7e-4)
            buf = []
            if time.perf_counter() >= deadline:
                break
    el = time.perf_counter() - t0
    if limiter is not None:
        limiter.unregister() if hasattr(limiter, "unregister") else None
    return {"value": steps / el, "unit": "env-steps/s", "cores": 1, "kind": "port", "steps": steps,
            "seconds": round(el, 3),
            "sample": f"{steps} env-steps ({steps // t_max} windows of t_max={t_max}) of one batch-1 "
                      f"A3C-FF actor-learner (NumPy restatement, 1 thread), {el:.1f} s"}


def _worker(args):
    seconds, t_max, n_actions, seed = args
    return run(seconds, t_max, n_actions, seed)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 CPU controller (cpu.max "quota period"),
    or None when unlimited / unreadable.  The GPU box runs a command under a
    16-CPU quota (cpu.max 1600000 100000) on a 128-core host: processes beyond
    the quota only time-share it."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota == "max":
            return None
        return max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def host_cores():
    """(physical cores, logical CPUs, CPUs this process may run on: the
    affinity mask, capped by the cgroup CPU quota)."""
    import os
    try:
        import psutil
        phys = psutil.cpu_count(logical=False)
    except Exception:  # pragma: no cover
        phys = None
    logical = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = logical
    quota = cgroup_cpu_quota()
    if quota is not None:
        avail = min(avail, quota)
    return phys or logical, logical, avail


def run_parallel(seconds: float = 10.0, t_max: int = 5, n_actions: int = 4, procs: int | None = None,
                 cap: int | None = None, ctx=None):
    """Leg (ii) of BASELINE.md §2: P independent actor-learner processes in
    the reference's style (async.py:68-90 run_async -- one process per
    core, OMP_NUM_THREADS=1 each, a3c_ale.py:186), P = min(physical cores,
    CPUs this process may use [, cap]).  "May use" includes the cgroup CPU
    quota: on the GPU box that is 16 CPUs of the 128-core host, so P = 16 is
    every core the bench can actually run on; more processes would only
    time-share those 16.  The record also states the per-process rate times
    the physical core count, labelled as an extrapolation (the reference's
    P = physical cores, run on the whole host).  Each process owns its
    parameters (the reference's shared RawArrays add Hogwild write traffic,
    not arithmetic).  Aggregate env-steps/s = sum of steps / the slowest
    process's time.  ctx: a multiprocessing context -- pass a forkserver
    started before the GPU was touched (bench.py) so no worker is forked
    from a GPU process."""
    import multiprocessing as mp
    phys, logical, avail = host_cores()
    P = procs if procs else max(1, min(phys, avail, cap or phys))
    ctx = ctx if ctx is not None else mp.get_context("forkserver")
    with ctx.Pool(P) as pool:
        res = pool.map(_worker, [(seconds, t_max, n_actions, 1000 + i) for i in range(P)])
    steps = [r["steps"] for r in res]
    rates = [r["value"] for r in res]
    el = max(r["seconds"] for r in res)
    per_proc = sum(rates) / len(rates)
    shared = (f"; {P} processes time-share the {avail} CPUs this process may use"
              if P > avail else "")
    return {"value": sum(steps) / el, "unit": "env-steps/s", "cores": P, "kind": "port",
            "sample": f"{P} processes x ~{seconds:.0f} s of the batch-1 A3C-FF actor-learner (NumPy restatement, "
                      f"1 thread each), {sum(steps)} env-steps in total; per-process {min(rates):.1f}-"
                      f"{max(rates):.1f} env-steps/s{shared}",
            "cpu_model": cpu_model(), "physical_cores": phys, "logical_cpus": logical, "cpus_allowed": avail,
            "cgroup_cpu_quota": cgroup_cpu_quota(),
            **({"extrapolated_physical_cores": {"value": round(per_proc * phys, 1), "cores": phys,
                                                "note": "mean per-process rate x physical cores: an estimate of "
                                                        "the reference-style P = physical-cores run on a whole "
                                                        "host, not a measurement (the quota admits only "
                                                        "cpus_allowed processes at once)"}}
               if P <= avail and P < phys else {})}


if __name__ == "__main__":
    print(run(5.0))
    print(run_parallel(5.0))
