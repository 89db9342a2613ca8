"""GPU: the bench's multi-rank launch and the RCCL path.

* `python bench.py --gpus 2` (no WORLD_SIZE) starts its two ranks itself
  (reference: run_async, async.py:68-90) -- gloo transport, both ranks on the
  one GPU of the box -- and reports n_gpus = ranks_seen = 2.
* `ARL_BENCH_FORCE_DIST=1 python bench.py --gpus 1` runs the N > 1 window
  (sectioned all-reduce around the conv backward, norm pass, eager
  collectives) over a one-rank RCCL process group.
* A one-rank RCCL group through A3C(collectives=True) gives the same update
  as the collective-free learner (tests/rccl_worker.py).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--workload", "c2", "--steps", "10", "--warmup", "3", "--cpu-seconds", "0", "--kernel-reps", "3", "--secondary", "none",
         "--median-windows", "20", "--copy-peak", "0"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.strip().splitlines() if ln.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def test_bench_starts_its_ranks(gpu):
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + SMALL, capture_output=True, text=True, timeout=300,
                       env=_env(ARL_BENCH_DIST_BACKEND="gloo", ARL_BENCH_SHARE_GPU="1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2, d
    assert d["collectives"] == "gloo"
    assert d["config"]["global_envs"] == 2 * d["config"]["envs_per_gpu"]
    assert d["allreduce_bytes_per_window"] >= 4 * 677429
    assert d["params_finite"] and d["windows"]["n"] == 20
    assert d["replicas_identical"] is True                                          # after the timed windows
    assert len([ln for ln in r.stdout.splitlines() if ln.startswith("{")]) == 1     # rank 0 only


def test_bench_rccl_one_rank(gpu):
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"] + SMALL, capture_output=True, text=True, timeout=300,
                       env=_env(ARL_BENCH_FORCE_DIST="1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1 and d["collectives"] == "rccl", d
    assert d["params_finite"]


def test_bench_window_timeline(gpu):
    """The per-stage table is the window's own, and every fraction in the line
    can fail: sparsely stamped eager windows of the default workload (C4, the
    driver's) give each stage's launches per window (phi T = 5, the forward
    stages T + 1, the learner's launches once); the RAW sparse shares (each
    carries one event's cost) add up to within 8 % of the unstamped window;
    with the measured copy peak on, no HBM stage exceeds the spec or the
    measured peak, and no MFMA stage exceeds the ceiling of the instructions it
    issues (frac, frac_issued <= 1)."""
    args = ["--steps", "10", "--warmup", "3", "--cpu-seconds", "0", "--kernel-reps", "3", "--secondary", "none",
            "--median-windows", "40", "--stamp-windows", "40"]
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"] + args, capture_output=True, text=True, timeout=300,
                       env=_env())
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _last_json(r.stdout)
    tl = d["timeline"]
    # (the returns run in the bootstrap step's policy launch: policy_fc_returns_kernel)
    want = {"phi": 5, "conv_fwd": 6, "fc_fwd": 6, "policy": 6, "fc_bwd": 1, "conv_bwd": 1, "conv_reduce": 1,
            "rmsprop": 1}
    assert {k: v["launches_per_window"] for k, v in tl["stages"].items()} == want, tl
    share = sum(v["window_share_us"] for v in tl["stages"].values())
    assert abs(share / 1e3 - tl["sum_of_shares_ms"]) <= 0.01 * tl["sum_of_shares_ms"], tl
    assert min(v["samples"] for v in tl["stages"].values()) >= 4, tl
    assert 0.97 <= tl["sum_vs_unstamped_median"] <= 1.08, tl
    peak = d["hbm_copy_peak"]["GB/s"]
    assert peak >= 6000, d["hbm_copy_peak"]
    for k, v in d["kernels"].items():
        if k not in want:
            continue
        assert v["time_source"] == "window", (k, v)
        assert v["frac"] <= 1.0 and v["standalone_frac"] <= 1.0, (k, v)
        if v["bound"] == "hbm":
            assert v["frac_measured_peak"] <= 1.0, (k, v)
        if v["bound"] == "mfma":
            assert v["issued"]["frac_issued"] <= 1.0 and v["issued"]["standalone_frac_issued"] <= 1.0, (k, v)
            assert v["frac"] <= v["issued"]["frac_issued"] + 1e-6, (k, v)   # padding only adds issued cycles
    ro = d["roofline"]
    assert ro["time_source"] == "window" and ro["frac"] <= 1.0 and ro.get("frac_issued", 0) <= 1.0, ro


def test_bench_secondary_workload(gpu):
    """--secondary: another BASELINE workload measured after the headline with
    the same protocol, reported beside it (the default line carries C3)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"] + SMALL + ["--secondary", "c2", "--stamp-windows", "0"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _last_json(r.stdout)
    (sec,) = d["secondary"]
    assert sec["workload"].startswith("c2") and sec["steps"] == 10 and sec["params_finite"], sec
    assert sec["value"] > 0 and sec["median_window_ms"] > 0


def test_bench_gpus_mismatch_fails(gpu):
    """A rank whose WORLD_SIZE disagrees with --gpus refuses to measure."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"] + SMALL, capture_output=True, text=True, timeout=300,
                       env=_env(WORLD_SIZE="1"))
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_rccl_collective_learner_matches_local(gpu, tmp_path):
    out = tmp_path / "res.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py"), str(out)],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["backend"] == "nccl"
    assert res["actions_equal"], res
    assert res["param_rel_err"] < 1e-6, res
    assert res["grad_rel_err"] < 1e-6, res
