"""Generates tests/golden/h5_fixture.h5 + h5_fixture_expected.npz with h5py
(run with an interpreter that has h5py, e.g. /opt/conda/bin/python3.9 in the
build container; not needed at test time).

The file uses the storage forms Chainer's save_hdf5 (h5py, compression=4)
produces for checkpoints (a3c.py:181-185) plus the others the reader
supports: gzip-chunked datasets with edge chunks, shuffle+gzip, contiguous,
compact, a scalar, big-endian and integer types, and a group with 300
children (multi-level group B-tree, many symbol nodes)."""
import os

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
rng = np.random.default_rng(2024)
exp = {}
with h5py.File(os.path.join(HERE, "h5_fixture.h5"), "w") as f:
    def put(path, arr, **kw):
        f.create_dataset(path, data=arr, **kw)
        exp[path] = np.asarray(arr).astype(np.asarray(arr).dtype.newbyteorder("="))

    put("0/0/W", rng.standard_normal((16, 4, 8, 8)).astype(np.float32), compression="gzip", compression_opts=4,
        chunks=(8, 4, 8, 8))
    put("0/0/b", rng.standard_normal(16).astype(np.float32), compression="gzip", compression_opts=4)
    put("0/2/W", rng.standard_normal((37, 53)).astype(np.float32), compression="gzip", compression_opts=4,
        chunks=(16, 20))                                     # edge chunks
    put("shuf", rng.standard_normal((100,)).astype(np.float64), compression="gzip", shuffle=True, chunks=(30,))
    put("contig", rng.integers(-5, 5, (7, 3)).astype(np.int32))
    put("compact", np.arange(5, dtype=np.int16), **{})
    f["compact_layout"] = np.arange(6, dtype=np.uint8)
    put("be", rng.standard_normal(9).astype(">f4"))
    put("t", np.array(123456789, np.int64))
    for i in range(300):
        put("many/d%03d" % i, np.array([i, -i], np.int64))
exp["compact_layout"] = np.arange(6, dtype=np.uint8)
np.savez(os.path.join(HERE, "h5_fixture_expected.npz"), **{k.replace("/", "|"): v for k, v in exp.items()})
print("wrote", len(exp), "datasets")
