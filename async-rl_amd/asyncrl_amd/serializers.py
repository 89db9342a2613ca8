"""Drop-in for the two `chainer.serializers` calls the reference makes:
`save_hdf5(filename, obj)` and `load_hdf5(filename, obj)` (a3c.py:169-185,
demo_a3c_ale.py:61), for obj = a model (A3CModel) or its RMSpropAsync.

File layout = Chainer 1.8.1's HDF5Serializer on these objects:
  model:      one dataset per parameter at its link path, "0/0/W", "0/0/b",
              ... (pinned by trained_model/breakout_ff/80000000_finish.h5,
              tests/test_checkpoint.py);
  optimizer:  scalars "t" and "epoch", then every parameter's state under
              its path, "0/0/W/ms", ... (Optimizer.serialize restated; no
              reference .opt file exists to pin it).
Reading accepts the chunked/deflated files h5py writes; writing produces
contiguous datasets (hdf5.py).  Host-side, off the hot path."""
from __future__ import annotations

import numpy as np
import torch

from .hdf5 import read_hdf5, write_hdf5


def _is_optimizer(obj) -> bool:
    return hasattr(obj, "target") and hasattr(obj, "hooks")


def state_arrays(obj) -> dict:
    if _is_optimizer(obj):
        net = obj.target.net
        out = {"t": np.array(int(getattr(obj, "t", 0)), np.int64), "epoch": np.array(int(getattr(obj, "epoch", 0)),
                                                                                       np.int64)}
        for name, a in net.state_dict(net.ms).items():
            out[name + "/ms"] = a
        return out
    return obj.net.state_dict()


def save_hdf5(filename, obj) -> None:
    """chainer.serializers.save_hdf5(filename, obj)."""
    write_hdf5(filename, state_arrays(obj))


def load_hdf5(filename, obj) -> None:
    """chainer.serializers.load_hdf5(filename, obj): every parameter (or
    optimizer state) of obj must be present with its shape; extra datasets
    are ignored, as Chainer's deserializer only visits obj's own entries."""
    data = read_hdf5(filename)
    if _is_optimizer(obj):
        net = obj.target.net
        obj.t = int(data["t"]) if "t" in data else 0
        obj.epoch = int(data["epoch"]) if "epoch" in data else 0
        for name, (_, shape) in net.layout.items():
            key = name + "/ms"
            if key not in data:
                raise KeyError("%s: no dataset %s" % (filename, key))
            net.view(net.ms, name).copy_(torch.from_numpy(np.asarray(data[key], np.float32).reshape(shape)))
        return
    net = obj.net
    missing = [n for n in net.layout if n not in data]
    if missing:
        raise KeyError("%s: missing parameters %s" % (filename, missing))
    for name, (_, shape) in net.layout.items():
        if tuple(data[name].shape) != tuple(shape):
            raise ValueError("%s: %s has shape %s, model expects %s" % (filename, name, data[name].shape, shape))
    net.load_params({n: data[n] for n in net.layout})
