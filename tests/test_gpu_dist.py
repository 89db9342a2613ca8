"""GPU: two env-sharded ranks (torch.distributed.run, gloo transport on one
GPU) keep bitwise-identical replicas and match the single-process learner
over the union of envs (same sampled actions; parameter deltas within 1e-4,
norm-scaled -- the gradient sum order differs)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_two_ranks_match_single_process(gpu, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "res.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "dist_gpu_worker.py"), str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert all(res["identical"]), res
    assert res["actions_equal"], res
    assert res["delta_rel_err"] < 1e-4, res
