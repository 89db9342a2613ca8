"""Chainer-HDF5 checkpoint I/O (a3c.py:169-185,
demo_a3c_ale.py:61): the pure-Python HDF5 reader against files written by
h5py (a committed fixture and, when present, the reference's trained
Breakout model), the writer against h5py and itself, and A3C.save_model /
load_model on the device."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, load_checkpoint

from asyncrl_amd.hdf5 import read_hdf5, write_hdf5

REF_H5 = "/root/reference/trained_model/breakout_ff/80000000_finish.h5"
CONDA_PY = "/opt/conda/bin/python3.9"


def test_reader_matches_h5py_fixture():
    """tests/golden/gen_h5_fixture.py (h5py 3.3 / HDF5 1.10): gzip chunks with
    edge chunks, shuffle, contiguous, big-endian, scalar, int types and a
    300-child group (multi-level B-tree)."""
    got = read_hdf5(os.path.join(GOLDEN, "h5_fixture.h5"))
    with np.load(os.path.join(GOLDEN, "h5_fixture_expected.npz")) as z:
        want = {k.replace("|", "/"): z[k] for k in z.files}
    assert set(got) == set(want)
    for k, v in want.items():
        assert got[k].dtype == v.dtype.newbyteorder("="), k
        assert got[k].shape == v.shape and (got[k] == v).all(), k


@pytest.mark.skipif(not os.path.exists(REF_H5), reason="reference checkpoint not present")
def test_reader_reads_reference_checkpoint():
    got = read_hdf5(REF_H5)
    want = load_checkpoint()
    assert set(got) == set(want)
    for k, v in want.items():
        assert got[k].dtype == np.float32 and (got[k] == v).all(), k


def _sample_arrays():
    rng = np.random.default_rng(3)
    arrs = dict(load_checkpoint())
    arrs["t"] = np.array(987654321, np.int64)
    arrs["epoch"] = np.array(0, np.int64)
    arrs["opt/1/0/W/ms"] = rng.random((4, 256)).astype(np.float32)
    for i in range(40):                      # > 2K symbol-node entries: several SNODs
        arrs["wide/k%02d" % i] = rng.integers(-9, 9, i % 5 + 1).astype(np.int32)
    arrs["f64"] = rng.standard_normal((2, 3, 4))
    arrs["u8"] = rng.integers(0, 255, 17).astype(np.uint8)
    arrs["empty"] = np.zeros((0, 3), np.float32)
    return arrs


def test_writer_roundtrip(tmp_path):
    arrs = _sample_arrays()
    fn = str(tmp_path / "m.h5")
    write_hdf5(fn, arrs)
    got = read_hdf5(fn)
    assert set(got) == set(arrs)
    for k, v in arrs.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape and (got[k] == v).all(), k


@pytest.mark.skipif(not os.path.exists(CONDA_PY), reason="no h5py interpreter in this container")
def test_writer_output_readable_by_h5py(tmp_path):
    arrs = _sample_arrays()
    fn = str(tmp_path / "m.h5")
    write_hdf5(fn, arrs)
    out = str(tmp_path / "back.npz")
    code = ("import h5py, numpy as np, sys\n"
            "f = h5py.File(sys.argv[1], 'r'); d = {}\n"
            "f.visititems(lambda n, o: d.__setitem__(n.replace('/', '|'), o[()]) "
            "if isinstance(o, h5py.Dataset) else None)\n"
            "np.savez(sys.argv[2], **d)\n")
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    subprocess.run([CONDA_PY, "-c", code, fn, out], check=True, env=env, timeout=120)
    with np.load(out) as z:
        got = {k.replace("|", "/"): z[k] for k in z.files}
    assert set(got) == set(arrs)
    for k, v in arrs.items():
        assert got[k].shape == v.shape and (got[k] == v).all(), k


def test_reader_rejects_non_hdf5(tmp_path):
    fn = tmp_path / "x.h5"
    fn.write_bytes(b"not an hdf5 file at all")
    with pytest.raises(ValueError):
        read_hdf5(str(fn))


@pytest.mark.gpu
def test_a3c_save_load_model_roundtrip(gpu, tmp_path):
    """A3C.save_model / load_model (a3c.py:169-185) through HDF5: the trained
    Breakout weights written as a Chainer-layout file load into the device
    model bit-exactly; a trained window's params and RMSProp state survive a
    save -> load into a fresh agent."""
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync, serializers
    from sim import make_pools
    ck = load_checkpoint()
    fn = str(tmp_path / "breakout.h5")
    write_hdf5(fn, ck)
    model = A3CFF(4, n_envs=4, t_max=5, init_seed=1)
    serializers.load_hdf5(fn, model)
    got = model.net.state_dict()
    assert all((got[k] == v).all() for k, v in ck.items())
    # one window of training, then save / load into a fresh agent
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(GradientClipping(40))
    agent = A3C(model, opt, 5, 0.99)
    pairs, rewards, dones = make_pools(np.random.default_rng(0), 6, 4, "uniform")
    t = lambda x: torch.from_numpy(x).to(gpu)  # noqa: E731
    agent.run_window(t(pairs), t(rewards), t(dones), 6, first=True)
    torch.cuda.synchronize()
    base = str(tmp_path / "agent.h5")
    agent.save_model(base)
    assert os.path.exists(base + ".opt")
    model2 = A3CFF(4, n_envs=4, t_max=5, init_seed=2)
    opt2 = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model2)
    agent2 = A3C(model2, opt2, 5, 0.99)
    agent2.load_model(base)
    p1, p2 = model.net.state_dict(), model2.net.state_dict()
    m1, m2 = model.net.state_dict(model.net.ms), model2.net.state_dict(model2.net.ms)
    assert all((p1[k] == p2[k]).all() and (m1[k] == m2[k]).all() for k in p1)
    assert opt2.t == opt.t == 1
    assert read_hdf5(base + ".opt")["0/2/W/ms"].shape == (256, 2592)
