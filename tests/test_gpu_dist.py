"""GPU: the N > 1 learner window (env-sharded ranks, torch.distributed.run,
gloo transport on the box's one GPU).

* test_two_rank_window_matches_oracle: the window the 8-GPU bench runs
  (collectives on, the gradient all-reduced in two sections around the conv
  backward, GradientClipping from grad_sqnorm on the reduced gradient, RMSProp)
  at 256 envs per rank against the oracle's f64 sum over both shards: the
  reduced gradient componentwise at 1e-5, the clip, the post-RMSProp
  parameters; replicas bitwise identical (tests/dist_window_worker.py).
* test_two_ranks_match_single_process: two ranks of 4 envs against one
  process over the union of 8 envs: bitwise-identical replicas, the same
  sampled actions, parameter deltas within 1e-5 norm-scaled (the gradient sum
  order differs; tests/dist_gpu_worker.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run2(worker, out, timeout=600):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", worker), str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_two_rank_window_matches_oracle(gpu, tmp_path):
    _run2("dist_window_worker.py", tmp_path)
    res = json.loads((tmp_path / "res.json").read_text())
    res1 = json.loads((tmp_path / "res1.json").read_text())
    assert res["world"] == 2 and res["envs_per_rank"] >= 256
    for win, win1 in zip(res["windows"], res1["windows"]):
        assert all(win["identical"].values()) and all(win1["identical"].values()), (win, win1)
        assert win["checksum_params"] == win1["checksum_params"]
        assert not win["grad_bad"], {k: (win["grad_err_normscaled"][k], win["grad_err_componentwise"][k])
                                     for k in win["grad_bad"]}
        assert win["clip_active"], win["norm_oracle"]
        assert win["norm_rel_err"] < 1e-5, win
        assert max(win["update_err_same_grad"]) <= 1e-5, win
        assert max(win["update_err_oracle_grad"]) <= 1e-5, win


def test_two_ranks_match_single_process(gpu, tmp_path):
    out = tmp_path / "res.json"
    _run2("dist_gpu_worker.py", out)
    res = json.loads(out.read_text())
    assert all(res["identical"]), res
    assert res["actions_equal"], res
    assert res["delta_rel_err"] < 1e-5, res
