"""CPU: the C-ABI library loads, exports every symbol include/asyncrl_hip.h
declares, and its host-side logic (layout, validation) behaves -- no kernel
launches (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "asyncrl_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(arl_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from asyncrl_amd import _lib
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(_lib.lib, s), s
    # and the ctypes table covers exactly the header
    assert sorted(_lib.SIGNATURES) == syms


def test_abi_version_and_errors():
    from asyncrl_amd._lib import lib
    assert lib.arl_abi_version() == 4
    h = ctypes.c_void_p()
    rc = lib.arl_net_create(ctypes.byref(h), 7, 4, 16, 5, 0, 0)
    assert rc == 1 and b"arch" in lib.arl_last_error()
    rc = lib.arl_net_create(ctypes.byref(h), 0, 0, 16, 5, 0, 0)
    assert rc == 1
    rc = lib.arl_net_create(ctypes.byref(h), 2 | 16, 4, 16, 5, 0, 0)   # Nature head has no RGB model
    assert rc == 1 and b"RGB" in lib.arl_last_error()
    for bad in (2 | 32, 16 | 32):                                        # STACK: NIPS FF / LSTM, not with RGB
        assert lib.arl_net_create(ctypes.byref(h), bad, 4, 16, 5, 0, 0) == 1
    # calls on an unbound handle fail cleanly
    assert lib.arl_net_create(ctypes.byref(h), 0, 4, 16, 5, 0, 0) == 0
    assert lib.arl_act(h, 0, None) == 3
    assert lib.arl_act(h, 0, None) == 3 and b"bound" in lib.arl_last_error()
    assert lib.arl_truncate_window(h, 2, None) == 3
    assert lib.arl_net_set_loss(h, 0.5, 1) == 0                          # host state only
    assert lib.arl_observe_stack(h, 0, None, None, None, 1, 0, None) == 3
    lib.arl_net_destroy(h)


# 16 / 17: the ViZDoom models (ARL_ARCH_RGB, train_a3c_doom.py:25-63), conv1 W (16, 3, 8, 8)
# 32 / 33: ARL_ARCH_STACK (whole ALE.state stacks per ring slot, the A3C.act drop-in)
@pytest.mark.parametrize("arch,A,count", [(0, 4, 677429), (1, 6, 1203255), (2, 4, 1686693),
                                          (16, 3, 676148), (17, 3, 1201460), (32, 4, 677429), (33, 6, 1203255)])
def test_param_layout_matches_chainer(arch, A, count):
    from asyncrl_amd._lib import lib
    from asyncrl_amd.net import param_shapes
    import numpy as np
    h = ctypes.c_void_p()
    assert lib.arl_net_create(ctypes.byref(h), arch, A, 256, 5, 0, 0) == 0
    shapes = param_shapes(arch, A)
    assert lib.arl_net_param_count(h) == len(shapes)
    name = ctypes.create_string_buffer(64)
    total = 0
    prev_end = 0
    for i, (nm, shp) in enumerate(shapes):
        off, num = ctypes.c_int64(), ctypes.c_int64()
        assert lib.arl_net_param_info(h, i, ctypes.byref(off), ctypes.byref(num), name, 64) == 0
        assert name.value.decode() == nm
        assert num.value == int(np.prod(shp))
        assert off.value % 64 == 0 and off.value >= prev_end
        prev_end = off.value + num.value
        total += num.value
    assert total == count
    assert lib.arl_net_param_floats(h) >= total
    ws = lib.arl_net_workspace_bytes(h)
    assert 0 < ws < 4 << 30
    off, nb = ctypes.c_int64(), ctypes.c_int64()
    assert lib.arl_net_buffer(h, b"frames", ctypes.byref(off), ctypes.byref(nb)) == 0
    assert nb.value == 9 * 256 * 84 * 84 * (3 if arch & 16 else 4 if arch & 32 else 1) and off.value % 256 == 0
    assert lib.arl_net_buffer(h, b"nope", ctypes.byref(off), ctypes.byref(nb)) == 1
    lib.arl_net_destroy(h)


def test_product_path_has_no_oracle_dependency():
    """The shipped package must never import the CPU oracle."""
    pkg = os.path.join(ROOT, "async-rl_amd", "asyncrl_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "oracle" not in src.replace("no oracle", ""), f


def test_env_group_split():
    """DeviceNet.env_groups: contiguous ranges, e0 a multiple of
    ENV_GROUP_ALIGN (the FC tile), covering every env exactly once; the
    Nature head never splits."""
    from types import SimpleNamespace
    from asyncrl_amd._lib import ARCH_FF, ARCH_FF_NATURE, ENV_GROUP_ALIGN
    from asyncrl_amd.net import DeviceNet
    for n in (1, 31, 32, 96, 100, 256, 1024):
        for g in (1, 2, 3, 4):
            rs = DeviceNet.env_groups(SimpleNamespace(n_envs=n, arch=ARCH_FF, states=False), g)
            assert rs[0][0] == 0 and sum(ne for _, ne in rs) == n and len(rs) <= g
            assert all(e0 % ENV_GROUP_ALIGN == 0 and ne > 0 for e0, ne in rs)
            assert all(rs[i][0] + rs[i][1] == rs[i + 1][0] for i in range(len(rs) - 1))
    assert DeviceNet.env_groups(SimpleNamespace(n_envs=256, arch=ARCH_FF, states=False), 2) == [(0, 128), (128, 128)]
    assert DeviceNet.env_groups(SimpleNamespace(n_envs=256, arch=ARCH_FF_NATURE), 2) == [(0, 256)]


def test_env_range_validation_without_device():
    """arl_observe_envs / arl_act_envs reject an unbound handle before any
    launch (no GPU needed)."""
    from asyncrl_amd._lib import lib
    h = ctypes.c_void_p()
    assert lib.arl_net_create(ctypes.byref(h), 0, 4, 64, 5, 0, 0) == 0
    try:
        assert lib.arl_act_envs(h, 0, 0, 32, 1, None) == 3        # ARL_ESTATE: not bound
        assert lib.arl_observe_envs(h, 0, 0, 32, None, 0, 0, None, None, 1, 0, 0, None) == 3
    finally:
        lib.arl_net_destroy(h)


def test_bench_launcher_propagates_rank_failure():
    """`python bench.py --gpus 2` without WORLD_SIZE starts two rank processes
    itself (bench.launch_ranks, the reference's run_async shape); when a rank
    fails -- here: no GPU in this container -- the launcher stops the other,
    reports it and exits non-zero instead of hanging."""
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--cpu-seconds", "0"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0
    assert "a rank failed" in r.stderr, r.stderr[-2000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_pool_len_checked_against_the_pools():
    """The C ABI sees only the pools' pointers: the Python mirror refuses a
    pool_len past any pool's leading dimension before a kernel could read past
    its buffer (a bench pass once handed pool_len 28 to an 8-entry pool)."""
    import torch
    from asyncrl_amd.net import check_pools
    pairs, rewards = torch.zeros(8, 2, 3, dtype=torch.uint8), torch.zeros(8, 2)
    check_pools(8, pairs, rewards, None)
    for bad in (0, 9, 28):
        with pytest.raises(ValueError):
            check_pools(bad, pairs, rewards, None)
    with pytest.raises(ValueError):
        check_pools(8, pairs, torch.zeros(4, 2))


def test_c_abi_rejects_pools_it_does_not_know():
    """The C ABI itself bounds every pool read (arl_net_set_pool): with fake,
    never-dereferenced device pointers on a bound handle, an unregistered pool
    and a pool_len past a registered pool's end fail with ARL_EINVAL before any
    launch -- arl_observe, arl_observe_envs and arl_run_window alike (no GPU
    needed: the checks run on the host)."""
    from asyncrl_amd._lib import POOL_DONES, POOL_FRAMES, POOL_REWARDS, lib
    N, T, PAIR = 4, 5, 2 * 210 * 160 * 3
    h = ctypes.c_void_p()
    assert lib.arl_net_create(ctypes.byref(h), 0, 4, N, T, 0, 0) == 0
    try:
        fake = 1 << 40                                   # 256-byte aligned, never dereferenced
        assert lib.arl_net_bind(h, fake, fake, fake, fake) == 0
        pairs, rew, done = fake + (1 << 30), fake + (2 << 30), fake + (3 << 30)
        EINVAL = 1
        # unregistered pools
        assert lib.arl_observe(h, 0, pairs, None, None, 8, 1, 0, None) == EINVAL
        assert b"not registered" in lib.arl_last_error()
        assert lib.arl_net_set_pool(h, 7, pairs, 64) == EINVAL        # unknown kind
        assert lib.arl_net_set_pool(h, POOL_FRAMES, pairs, 8 * N * PAIR) == 0
        assert lib.arl_net_set_pool(h, POOL_REWARDS, rew, 8 * N * 4) == 0
        assert lib.arl_net_set_pool(h, POOL_DONES, done, 8 * N) == 0
        # pool_len past a registered pool's end: refused, nothing launched
        for call in (lambda L: lib.arl_observe(h, 1, pairs, rew, done, L, 0, 0, None),
                     lambda L: lib.arl_observe_envs(h, 1, 0, N, pairs, 0, 0, rew, done, L, 0, 0, None),
                     lambda L: lib.arl_run_window(h, pairs, rew, done, L, 1, 0, 0.99, 0.01, 0.5, 1, 7e-4, 0, 0,
                                                  0.99, 0.1, 40.0, None)):
            for bad in (9, 28):
                assert call(bad) == EINVAL, bad
                assert b"exceeds" in lib.arl_last_error()
        # an interior pointer is checked against the room left before the pool's end
        assert lib.arl_observe(h, 1, pairs + 4 * N * PAIR, rew, done, 5, 0, 0, None) == EINVAL
        # a reward pool shorter than the frame pool
        assert lib.arl_net_set_pool(h, POOL_REWARDS, rew, 4 * N * 4) == 0   # re-registered smaller
        assert lib.arl_observe(h, 1, pairs, rew, done, 8, 0, 0, None) == EINVAL
        assert b"reward" in lib.arl_last_error()
        assert lib.arl_net_set_pool(h, POOL_REWARDS, rew, 0) == 0           # removed
        assert lib.arl_observe(h, 1, pairs, rew, done, 1, 0, 0, None) == EINVAL
        # a freed pool's stale, larger registration must not lend its room to a newer, smaller
        # pool allocated inside it -- registering the new pool drops every overlapping registration
        big, small = fake + (4 << 30), fake + (4 << 30) + 2 * N * PAIR
        assert lib.arl_net_set_pool(h, POOL_REWARDS, rew, 8 * N * 4) == 0
        assert lib.arl_net_set_pool(h, POOL_FRAMES, big, 8 * N * PAIR) == 0
        assert lib.arl_net_set_pool(h, POOL_FRAMES, small, 2 * N * PAIR) == 0   # (big freed, memory reused)
        assert lib.arl_observe(h, 1, small, rew, done, 3, 0, 0, None) == EINVAL
        assert b"exceeds" in lib.arl_last_error()
        assert lib.arl_observe(h, 1, big, rew, done, 1, 0, 0, None) == EINVAL  # the stale one is gone
        assert b"not registered" in lib.arl_last_error()
    finally:
        lib.arl_net_destroy(h)


def test_param_generation_without_device():
    """ABI 4 parameter generations on a bound handle (fake, never-dereferenced pointers; no launch):
    binding and arl_net_params_changed bump param_gen; the FC planes are stale until a forward or
    arl_net_prepare rebuilds them, so an env-range act refuses to run."""
    from asyncrl_amd._lib import lib
    h = ctypes.c_void_p()
    assert lib.arl_net_create(ctypes.byref(h), 0, 4, 64, 5, 0, 0) == 0
    try:
        pg, pl = ctypes.c_uint64(), ctypes.c_uint64()
        assert lib.arl_net_param_generation(h, ctypes.byref(pg), ctypes.byref(pl)) == 0
        g0 = pg.value
        fake = 1 << 40
        assert lib.arl_net_bind(h, fake, fake, fake, fake) == 0
        assert lib.arl_net_param_generation(h, ctypes.byref(pg), ctypes.byref(pl)) == 0
        assert pg.value == g0 + 1 and pl.value != pg.value
        assert lib.arl_net_params_changed(h) == 0
        assert lib.arl_net_param_generation(h, ctypes.byref(pg), None) == 0 and pg.value == g0 + 2
        assert lib.arl_act_envs(h, 0, 0, 32, 1, None) == 3                     # ARL_ESTATE: stale planes
        assert b"arl_net_prepare" in lib.arl_last_error()
    finally:
        lib.arl_net_destroy(h)
