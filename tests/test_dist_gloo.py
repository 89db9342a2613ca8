"""CPU, world_size 2 over gloo: the env-sharded learner's exchange.

Each rank computes the oracle gradient of ITS env shard at shared theta,
the package's allreduce_grads sums them, and the result must equal the
single-process gradient over all envs; the Philox streams keyed by global
env id must reproduce the single-process draws; replicas stay identical."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, close_normscaled


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (os.path.join(ROOT, "async-rl_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import oracle as O
    from asyncrl_amd.distributed import allreduce_grads, replicas_identical, shard_envs
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(5)
        T, G, A = 3, 6, 4
        params = O.init_like_torch(O.ARCH_FF, A, rng)
        states = O.PHI_LUT[rng.integers(0, 256, (T, G, 4, 84, 84), dtype=np.uint8)]
        boot = O.PHI_LUT[rng.integers(0, 256, (G, 4, 84, 84), dtype=np.uint8)]
        actions = rng.integers(0, A, (T, G)).astype(np.int32)
        rewards = rng.choice([-1.0, 0.0, 1.0], (T, G)).astype(np.float32)
        dones = (rng.random((T, G)) < 0.2).astype(np.uint8)
        n, off = shard_envs(G, world, rank)
        sl = slice(off, off + n)
        g_loc, _ = O.ff_window_grads(params, states[:, sl], actions[:, sl], rewards[:, sl], dones[:, sl], boot[sl])
        names = list(g_loc)
        flat = torch.from_numpy(np.concatenate([g_loc[k].ravel() for k in names]))
        allreduce_grads(flat)
        g_all, _ = O.ff_window_grads(params, states, actions, rewards, dones, boot)
        ref = np.concatenate([g_all[k].ravel() for k in names])
        ok, err = close_normscaled(flat.numpy(), ref, 1e-5)
        u_loc = O.sample_uniforms(99, np.arange(off, off + n, dtype=np.uint64), 17)
        u_all = O.sample_uniforms(99, np.arange(G, dtype=np.uint64), 17)
        rng_ok = bool((u_loc == u_all[sl]).all())
        same = replicas_identical(flat)
        q.put((rank, ok, err, rng_ok, same))
    finally:
        dist.destroy_process_group()


def test_two_rank_gradient_allreduce_equals_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, err, rng_ok, same in res:
        assert ok, (rank, err)
        assert rng_ok and same, rank


def test_shard_envs():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
    from asyncrl_amd.distributed import shard_envs
    assert shard_envs(4096, 8, 3) == (512, 1536)
    with pytest.raises(ValueError):
        shard_envs(10, 4, 0)


def _sections_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "async-rl_amd"))
    from asyncrl_amd.distributed import allreduce_grads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.from_numpy(np.random.default_rng(10 + rank).standard_normal(10_000).astype(np.float32))
        whole = g.clone()
        allreduce_grads(whole)
        o = 1_234                                    # conv section [0, o), the rest overlapped
        work = allreduce_grads(g[o:], async_op=True)
        assert work is not None
        work.wait()
        assert allreduce_grads(g[:o]) is None        # synchronous form returns nothing
        q.put((rank, bool(torch.equal(g, whole))))
    finally:
        dist.destroy_process_group()


def test_sectioned_allreduce_equals_whole():
    """A3C._reduce_and_step's split all-reduce (async FC / heads section,
    then the conv section) sums exactly like one all-reduce of the flat
    gradient (gloo, world_size 2)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sections_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
