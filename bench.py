"""Throughput of the batched A3C hot path (phi + forward + sample + n-step
update) on MI355X -- BASELINE.json metric.  Default workload: configs[3]'s
per-GPU leg (C4: A3C-FF, 512 envs per GPU), so `--gpus 8` IS configs[3]
(4096 envs over 8 GPUs, RCCL all-reduce) and the N=1 line is its
weak-scaling unit; `--workload c2|c3|c5` selects the other configs.

One bench *step* = one lockstep window: t_max x (phi of every env's frame
pair into the ring, NIPS-head forward, softmax policy, Philox sample), the
bootstrap phi + forward, n-step returns + loss gradient, backward, [RCCL
all-reduce of the flat gradient over ranks], GradientClipping(40) +
RMSpropAsync, advance.  Units = envs_per_gpu * t_max * world env-steps per
step.  Inputs are synthetic 210x160x3 RGB frame pairs, rewards and terminal
flags pre-generated in HBM (a pool of `--pool` steps, cycled).

    python bench.py [--gpus N] [--steps K] [--warmup W]
        --gpus N > 1 without WORLD_SIZE in the environment: this process starts
        N ranks itself (one child process per GPU, like the reference's
        run_async, async.py:68-90), touches no GPU, forwards rank 0's line.
    torchrun --nproc-per-node N bench.py --gpus N ...   (the same ranks, started by torchrun)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
# ASYNCRL_PKG_ROOT: another build of the package (A/B timing, scripts/ab.sh)
PKG_ROOT = os.environ.get("ASYNCRL_PKG_ROOT") or os.path.join(ROOT, "async-rl_amd")


def _import_pkg():
    """The package loads libasyncrl_hip.so (its code objects register with
    the HIP runtime): only rank processes import it, never the launcher."""
    sys.path.insert(0, PKG_ROOT)
    import asyncrl_amd
    return asyncrl_amd

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
F32_MFMA_PEAK_TFS = 157.3      # dense fp32 matrix peak (spec)
# The matrix pipe the kernels issue to (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs at the 2.4 GHz peak engine
# clock; v_mfma_f32_16x16x32_bf16 holds a SIMD's pipe 16 cycles (16,384 FLOP: the 2.5 PFLOP/s dense bf16
# peak), v_mfma_f32_16x16x4_f32 32 cycles (2,048 FLOP: the 157.3 TFLOP/s dense f32 peak).  An f32 product
# on exact bf16 splits costs 3 (pixel x f32) or 6 (f32 x f32) bf16 MFMAs (bf16split.hpp).
SIMDS, CLK_HZ = 1024, 2.4e9
BF16_CYC, F32_CYC = 16, 32
PHI_BYTES_PER_ENV_STEP = 201600 + 7056      # pair read + plane write (ring)
RMSPROP_BYTES_PER_PARAM = 20                # r p,g,ms; w p,ms
# algorithmic FLOPs (2 per MAC) per env / per sample, NIPS head
CONV_FWD_FLOP_PER_ENV = 2 * (400 * 16 * 256 + 81 * 32 * 256)             # 4,603,904
FC_FWD_FLOP_PER_ENV = 2 * 2592 * 256                                     # 1,327,104
CONV_BWD_FLOP_PER_SAMPLE = 2 * (32 * 256 * 81 + 81 * 32 * 256 + 400 * 16 * 256)   # dW2 + convT + dW1
HID_BYTES = 256 * 4
FC_SPLIT = 8                                # fc.hip split-K (partial slabs read by policy_fc_kernel)
# LSTM (a3c_ale.py:50-51,62; L.LSTM(256, 256)): gates = [x | h] [Wu ; Wl]^T (K = 512, N = 1024);
# BPTT dh = dG Wl (K = 1024, N = 256); gate weight gradients [x | h | 1]^T dG (513 x 1024 per
# sample) + dfc = dG Wu (K = 1024, N = 256)
LSTM_GATES_FLOP_PER_ENV = 2 * 512 * 1024
LSTM_BPTT_FLOP_PER_ENV = 2 * 1024 * 256
LSTM_WGRAD_FLOP_PER_SAMPLE = 2 * 513 * 1024 + 2 * 1024 * 256
# the LSTM gate kernel forms x from the FC's split-K partials (XRED) for launches under 512 envs, the
# FC's ticket reduce does from 512 up (net.hip lstm_xred); ARL_LSTM_XRED=1 / 0 forces one
def lstm_xred(n_launch):
    v = os.environ.get("ARL_LSTM_XRED", "")[:1]
    return v != "0" if v in ("0", "1") else n_launch < 512
# ViZDoom models (train_a3c_doom.py:28,46): conv1 K = 3 * 64 (the kernels' zero input plane is not counted)
DOOM_CONV_FWD_FLOP_PER_ENV = 2 * (400 * 16 * 192 + 81 * 32 * 256)
DOOM_CONV_BWD_FLOP_PER_SAMPLE = 2 * (32 * 256 * 81 + 81 * 32 * 256 + 400 * 16 * 192)
# NatureDQNHead (dqn_head.py:6-28): conv MACs 400*32*256 + 81*64*512 + 49*64*576, FC 3136*512
NAT_CONV_FWD_FLOP_PER_ENV = 2 * (400 * 32 * 256 + 81 * 64 * 512 + 49 * 64 * 576)      # 15,474,688
NAT_FC_FWD_FLOP_PER_ENV = 2 * 3136 * 512
NAT_CONV_BWD_FLOP_PER_SAMPLE = 2 * (2 * 49 * 64 * 576 + 2 * 81 * 64 * 512 + 400 * 32 * 256)
PHI_STACK_BYTES_PER_PAIR = 201600 + 3 * 7056 + 4 * 7056   # pair + 3 prior planes + 4-plane stack
PLANE_BYTES, A1_FLOATS, A2_FLOATS = 7056, 6400, 2592     # ring plane; conv1 / conv2 activations kept for backward
PHI_TAP_ROWS = 168          # source rows (of 210) the 84-row bilinear resize reads (phi.hip phi_band)

# BASELINE.json configs[1..4] -> (arch, envs per GPU, actions)
WORKLOADS = {"c2": ("ff", 256, 4), "c3": ("lstm", 1024, 6), "c4": ("ff", 512, 4), "c5": ("phi", 16384, 0)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c4",
                    help="BASELINE.json configs: c4 FF 512 envs per GPU (default: 4096 over 8 GPUs, the north-star "
                         "target's config), c2 FF 256 envs, c3 LSTM 1024 envs A=6, c5 phi stress 16384 frame pairs")
    ap.add_argument("--median-windows", type=int, default=200,
                    help="after the timed region: this many more windows, each between two HIP events on the "
                         "bench stream, for the per-window median / p10 / p90 (SURVEY 8(d)); 0 disables")
    ap.add_argument("--copy-peak", type=int, default=1, help="1: measure the HBM stream-copy peak on this GPU")
    ap.add_argument("--envs-per-gpu", type=int, default=0, help="0: the workload's")
    ap.add_argument("--t-max", type=int, default=5)
    ap.add_argument("--arch", choices=["ff", "lstm", "nature", "doom_ff", "doom_lstm"], default=None,
                    help="default: the workload's; nature = A3CFF with NatureDQNHead (SURVEY 8(a) a8); doom_* = "
                         "the ViZDoom models of train_a3c_doom.py on RGB screens (--doom-width)")
    ap.add_argument("--doom-width", type=int, choices=[160, 320, 640], default=640,
                    help="ViZDoom screen resolution (doom_env.py:43-46; 640 = 640x480, the default)")
    ap.add_argument("--actions", type=int, default=0, help="0: 4 for ff (Breakout), 6 for lstm (Space Invaders)")
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="window as one HIP graph replay or eager launches on one stream. auto: eager for a "
                         "one-chain window (C4 0.503-0.504 vs 0.510-0.512 ms median, C2 0.313-0.316 vs "
                         "0.318-0.320, the N > 1 window on a one-rank RCCL group 0.547-0.550 vs 0.561-0.565; "
                         "profiles/r03/r3ag, r3am), the graph for env-group chains (C3)")
    ap.add_argument("--no-graph", action="store_true", help="= --graph off")
    ap.add_argument("--env-groups", type=int, default=0,
                    help="forward chains on separate streams per window (A3C.run_window env_groups); "
                         "0: the library default (2 from 1,024 envs per GPU up, else 1)")
    ap.add_argument("--stamp-windows", type=int, default=100,
                    help="after the median windows: this many eager windows with a HIP event after every stage "
                         "launch (arl_stamps_*), whose intervals give each stage's in-window time and share; 0 "
                         "disables (the per-stage table then falls back to standalone relaunches)")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="> 1 rank: torch.distributed timeout (s); a rank stuck in a collective raises and the "
                         "launcher exits non-zero")
    ap.add_argument("--secondary", default="auto",
                    help="comma-separated BASELINE workloads (c2, c3) also measured on one GPU after the headline, "
                         "with the same protocol (W warmup, K timed windows, median over 100), reported under "
                         "'secondary'; auto: c3 beside the default c4 line at N = 1; none disables")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="0 disables the CPU baseline leg")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--timed-diag", type=int, default=0,
                    help="diagnostic (off by default): after the timed region, repeat its shape (sync, K windows, "
                         "sync) this many times with a HIP event after every window, to attribute the gap between "
                         "the timed mean and the per-window median (first window vs the rest, host edges)")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` (N > 1) run as a plain `python bench.py`: start the N rank
    processes here, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1), the way the reference's run_async starts its
    actor-learners (async.py:68-90).  This process never touches the GPU (no
    torch.cuda call, no import of the HIP extension) and never execs: it
    waits for the children, which inherit stdout (rank 0 prints the line),
    and exits with the first failing child's status after stopping the rest
    (a rank left alone would wait in a collective forever)."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    # a whole-run deadline on top of the ranks' collective timeout: a rank that hangs outside a
    # collective (e.g. in a kernel) would otherwise hold the run (and its peers) forever
    deadline_s = float(os.environ.get("ARL_BENCH_DEADLINE_S", "1800"))
    t_start = time.time()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if time.time() - t_start > deadline_s:
                print(f"bench.py: ranks still running after {deadline_s:.0f} s (ARL_BENCH_DEADLINE_S); stopping them",
                      file=sys.stderr)
                rc = 124
                break
            time.sleep(0.1)
    finally:
        rc = rc or next((p.returncode for p in procs if p.returncode not in (None, 0)), 0)
        if rc:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + 10
            for p in procs:
                try:
                    p.wait(max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    if rc:
        print(f"bench.py: a rank failed (status {rc})", file=sys.stderr)
    return 0 if rc == 0 else (rc if rc > 0 else 1)


CONV_SLAB_FLOATS = 12336                    # conv_slab.hpp SLAB: one conv_bwd workgroup's partial gradient


def conv_bwd_blocks(S):
    """conv_bwd.hip conv_bwd_blocks: slab slices of the conv backward."""
    g0 = min(S, 256)
    spb = -(-S // g0)
    return -(-S // spb)


def returns_bytes(N, T, A, mask=True, hid=256):
    """Algorithmic bytes of the learner's first launch (policy.hip
    returns_heads_kernel): read rewards, dones, v (T + 1 rows), probs, logp,
    actions, [the h > 0 mask], the heads' weights; write dlogits, dv, the
    per-env losses and dh."""
    S = N * T
    return (S * (4 + 1 + 4 + 8 * A + 4) + 4 * N + (A + 1) * hid * 4 + (S * hid * 4 if mask else 0)
            + S * (4 * A + 4) + 8 * N + S * hid * 4)


def conv_epw(n_envs):
    """Envs per conv_fwd workgroup the library picks for a net of n_envs
    (conv_fwd.hip launch_conv_fwd: two from 512 envs; ARL_CONV_EPW forces)."""
    v = os.environ.get("ARL_CONV_EPW", "")[:1]
    return int(v) if v in ("1", "2") else (2 if n_envs >= 512 else 1)


def fc_big(n_launch):
    """fc.hip launch_fc_fwd: 64-row tiles (fc_fwd_big_kernel) for partials-only
    launches over >= 512 envs; ARL_FC_BIG forces."""
    v = os.environ.get("ARL_FC_BIG", "")[:1]
    return v == "1" if v in ("0", "1") else n_launch >= 512


def _cdiv(a, b):
    return -(-a // b)


def fc_bwd_ranges(S, lstm=False):
    """fc_bwd.hip fc_bwd_ranges / lstm_wgrad_ranges and range_len: job A's sample ranges."""
    Z = max(1, min(16, (S + 400) // 800))
    if lstm:
        Z = max(Z, _cdiv(S, 1024))
    kpz = _cdiv(_cdiv(S, Z), 32) * 32
    return [min(S, (z + 1) * kpz) - z * kpz for z in range(Z) if z * kpz < S]


def mfma_cycles(stage, N, T, arch="ff"):
    """Matrix-pipe cycles one launch of `stage` issues (the instruction counts
    of the kernel as written, padding included), summed over SIMDs; None for
    stages without MFMAs.  Divided by SIMDS x CLK_HZ x the launch time this is
    the fraction of the chip's matrix pipe the launch keeps busy -- the model
    of SQ_VALU_MFMA_BUSY_CYCLES (scripts/mfma_util.py checks it against the
    counter)."""
    S = N * T
    if stage == "conv_fwd":   # conv_fwd.hip: conv1 25 position tiles x 8 k-steps x 3 (mfma_x3_t); conv2 6 x 2
        return N * (25 * 8 * 3 + 6 * 2 * 8 * 6) * BF16_CYC   # tiles x 8 k-steps x 6 (mfma_x6_t)
    if stage == "fc_fwd":     # fc.hip: 16 x 16 sub-tiles x 8 K slices (324 k): 10 split k-steps x 6
        rows = _cdiv(N, 64) * 64 if fc_big(N) else _cdiv(N, 32) * 32   # (mfma_x6) + one f32 16x16x4 tail
        return (rows // 16) * (256 // 16) * 8 * (10 * 6 * BF16_CYC + F32_CYC)
    if stage in ("fc_bwd", "lstm_wgrad"):   # fc_bwd.hip: job A 4 waves x (4 x 2 tile pairs x 6) per 32-sample
        lstm = stage == "lstm_wgrad"         # chunk of each range; job B 4 waves x (2 x 4 x 6) per 32-j chunk
        nta = (1024 // 128) * (512 // 64) if lstm else (256 // 128) * _cdiv(2592, 64)
        chunks = sum(_cdiv(r, 32) for r in fc_bwd_ranges(S, lstm))
        job_a = nta * chunks * 4 * 48
        job_b = _cdiv(S, 64) * (_cdiv(256, 128) if lstm else _cdiv(2592, 128)) * (1024 // 32 if lstm else 256 // 32) * 4 * 48
        return (job_a + job_b) * BF16_CYC
    if stage == "conv_bwd":   # conv_bwd.hip per sample, 6-term (mfma_x6) / 3-term (mfma_x3) splits:
        # (1) 8 waves x 3 k-steps x 2 x 2 tiles x 6; (2) 28 tiles x 4 k-steps x 6; (3) 8 waves x 15 x 2 x 3
        return S * (8 * 3 * 4 * 6 + 28 * 4 * 6 + 8 * 15 * 2 * 3) * BF16_CYC
    if stage == "lstm_gates":  # lstm.hip: 32-row tiles, K = 512 on f32 16x16x4
        return _cdiv(N, 32) * 32 * 1024 * 512 * 2 // 64
    if stage == "lstm_bptt":   # lstm.hip: 32-row tiles, N = 256, K = 1024 on f32 16x16x4
        return _cdiv(N, 32) * 32 * 256 * 1024 * 2 // 64
    return None


def mfma_ideal_cycles(stage, N, T):
    """The same contractions' algorithmic FLOPs at the rate of the instructions
    they run on, no padding (the f32-equivalent ceiling of the kernel's
    instruction mix: bf16 2.5 PFLOP/s / 3 or / 6 terms, exact f32 157.3)."""
    S = N * T
    b3, b6, f = 3 / 1024, 6 / 1024, 1 / 64   # cycles per FLOP
    if stage == "conv_fwd":
        return N * (2 * 400 * 16 * 256 * b3 + 2 * 81 * 32 * 256 * b6)
    if stage == "fc_fwd":   # 320 of each K slice's 324 k on the split, the last 4 on f32
        return N * FC_FWD_FLOP_PER_ENV * (320 * b6 + 4 * f) / 324
    if stage == "fc_bwd":
        return 2 * S * FC_FWD_FLOP_PER_ENV * b6
    if stage == "conv_bwd":
        return S * (2 * 32 * 256 * 81 * b6 + 2 * 81 * 32 * 256 * b6 + 2 * 400 * 16 * 256 * b3)
    if stage == "lstm_gates":
        return N * LSTM_GATES_FLOP_PER_ENV * f
    if stage == "lstm_bptt":
        return N * LSTM_BPTT_FLOP_PER_ENV * f
    if stage == "lstm_wgrad":
        return S * LSTM_WGRAD_FLOP_PER_SAMPLE * b6
    return None


def source_version():
    """Digest of the HIP sources and the C-ABI header: PMC traffic files
    record the version they were measured on, and the bench uses one only
    when it matches the tree it runs."""
    import glob
    import hashlib
    h = hashlib.sha1()
    files = sorted(glob.glob(os.path.join(ROOT, "async-rl_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "async-rl_amd", "csrc", "*.hpp")) +
                   glob.glob(os.path.join(ROOT, "include", "*.h")))
    for fn in files:
        with open(fn, "rb") as f:
            h.update(os.path.basename(fn).encode() + b"\0" + f.read())
    return h.hexdigest()[:12]


def measured_traffic(N, T, arch, kernel):
    """HBM bytes per dispatch of `kernel` from a profiles/traffic_*.json
    measured on this source version at this config (scripts/traffic.py), else None."""
    import glob
    ver = source_version()
    for tf in sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_*.json"))):
        try:
            with open(tf) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            continue
        if (tj.get("source_version") == ver and tj.get("envs") == N and tj.get("t_max") == T
                and tj.get("arch") == arch and kernel in tj.get("kernels", {})):
            return tj["kernels"][kernel]
    return None


def init_dist(timeout_s: float = 300.0):
    from datetime import timedelta
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a 1-GPU box: ARL_BENCH_DIST_BACKEND=gloo
    # ARL_BENCH_SHARE_GPU=1 puts every rank on cuda:0 (RCCL needs one GPU per rank)
    backend = os.environ.get("ARL_BENCH_DIST_BACKEND", "nccl")
    if os.environ.get("ARL_BENCH_SHARE_GPU") == "1":
        local = 0
    # ARL_BENCH_FORCE_DIST=1 at one rank: a one-rank process group and the full
    # N > 1 window (sectioned all-reduce around the conv backward, eager
    # collectives, the norm pass) -- the RCCL calls rehearsed on one GPU
    force = os.environ.get("ARL_BENCH_FORCE_DIST") == "1"
    torch.cuda.set_device(local)
    if world > 1 or force:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # a timeout so a rank stuck in a collective raises (RCCL's watchdog aborts it) and exits non-zero
        to = timedelta(seconds=timeout_s)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=to)
        else:
            dist.init_process_group(backend, timeout=to)
    return world, rank, local, (world > 1 or force)


def measure_copy_peak(dev, mib: int = 1024, reps: int = 10):
    """HBM stream-copy rate on this GPU (arl_stream_copy, every form: grid-
    stride with four 16-byte loads in flight per lane, 64 KB blocks per
    workgroup with non-temporal accesses, and a one-shot grid of one 16-byte
    load + store a lane, default-policy / non-temporal): a 1 GiB buffer
    (4x the 256 MiB Infinity Cache) copied `reps` times per form and grid
    size; the best one's read + write bytes / time."""
    from asyncrl_amd._lib import check, lib, ptr
    n = mib << 20
    src = torch.ones(n // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    s = torch.cuda.current_stream(dev)
    best, best_cfg, tried = 0.0, None, {}
    forms = {0: "gridstride", 1: "blocks64k_nt", 2: "oneshot", 3: "oneshot_nt"}
    for mode in (0, 1, 2, 3):
        for blocks in ((4096, 8192) if mode < 2 else (0,)):
            for _ in range(2):
                check(lib.arl_stream_copy(ptr(src), ptr(dst), n, blocks, mode, s.cuda_stream), "arl_stream_copy")
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(s)
            for _ in range(reps):
                check(lib.arl_stream_copy(ptr(src), ptr(dst), n, blocks, mode, s.cuda_stream), "arl_stream_copy")
            ev1.record(s)
            ev1.synchronize()
            gbs = 2 * n * reps / (ev0.elapsed_time(ev1) * 1e-3) / 1e9
            tried["%s/%d" % (forms[mode], blocks)] = round(gbs, 1)
            if gbs > best:
                best, best_cfg = gbs, (mode, blocks)
    ok = bool(torch.equal(src, dst))
    del src, dst
    torch.cuda.empty_cache()
    return {"GB/s": round(best, 1), "frac_of_spec": round(best / HBM_PEAK_GBS, 4), "bytes_per_copy": 2 * n,
            "kernel": {0: "stream_copy_kernel", 1: "stream_copy_blocks_kernel", 2: "stream_copy_chunk_kernel<false>",
                       3: "stream_copy_chunk_kernel<true>"}[best_cfg[0]] + " (optim.hip)",
            "blocks": best_cfg[1], "tried_GBs": tried, "copy_verified": ok}


def ranks_seen(dev) -> int:
    """Ranks that took part in a SUM all-reduce of ones over the bench's
    process group (the transport the gradient all-reduce uses)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    t = torch.ones(1, dtype=torch.float32, device=dev)
    dist.all_reduce(t)
    return int(round(float(t.item())))


def rgb_phi_bytes(H, W):
    """Algorithmic bytes of one ViZDoom observation (train_a3c_doom.py:21-23 into
    the ring): the distinct source rows the bilinear taps touch (OpenCV
    half-pixel mapping, 2 taps per output row) x W x 3, plus 3 planes written."""
    rows = set()
    for d in range(84):
        f = np.float32((d + 0.5) * (H / 84.0) - 0.5)
        s = max(0, min(int(np.floor(f)), H - 1))
        rows.update((s, min(s + 1, H - 1)))
    return len(rows) * W * 3 + 3 * 84 * 84


def synth_rgb_pools(n, pool, seed, dev, H, W):
    """ViZDoom-shaped synthetic inputs: uniform RGB24 screens (H, W, 3), rewards
    and terminals as synth_pools."""
    g = torch.Generator(device=dev)
    g.manual_seed(1 + 1000 * seed)
    imgs = torch.randint(0, 256, (pool, n, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    _, rewards, dones = synth_pools(n, 1, seed, dev, frames=False, pool_rd=pool)
    return imgs, rewards, dones


def synth_pools(n, pool, seed, dev, frames=True, pool_rd=None):
    """SURVEY 8(d) synthetic inputs: uniform RGB frames (rng 1), rewards in
    {-1,0,+1} with P(!=0)=0.05 (rng 2), terminals Bernoulli(1/500) (rng 3)."""
    g = torch.Generator(device=dev)
    g.manual_seed(1 + 1000 * seed)
    pairs = torch.randint(0, 256, (pool, n, 2, 210, 160, 3), dtype=torch.uint8, device=dev, generator=g) \
        if frames else None
    pool = pool_rd or pool
    r2 = np.random.default_rng(2 + 1000 * seed)
    rewards = r2.choice(np.array([-1.0, 0.0, 1.0], np.float32), (pool, n), p=[0.025, 0.95, 0.025])
    r3 = np.random.default_rng(3 + 1000 * seed)
    dones = (r3.random((pool, n)) < 1 / 500).astype(np.uint8)
    return pairs, torch.from_numpy(rewards).to(dev), torch.from_numpy(dones).to(dev)


def bench_phi(a, world, rank, dev, n_default, copy_peak=None):
    """configs[4] (c5): dqn_phi preprocessing stress -- one step = one batch of
    n frame pairs 210x160 RGB -> max -> luminance -> 84x84 -> 4-plane stack
    (arl_phi_stack, materialised), ping-pong stacks, reset flags from rng(3).
    Units = frame pairs (= env-steps of the phi stage)."""
    from asyncrl_amd.dqn_phi import phi_stack
    n = a.envs_per_gpu or n_default
    g = torch.Generator(device=dev)
    g.manual_seed(1 + 1000 * rank)
    pairs = torch.randint(0, 256, (n, 2, 210, 160, 3), dtype=torch.uint8, device=dev, generator=g)
    stacks = [torch.zeros((n, 4, 84, 84), dtype=torch.uint8, device=dev) for _ in range(2)]
    reset = torch.from_numpy((np.random.default_rng(3 + 1000 * rank).random(n) < 1 / 500).astype(np.uint8)).to(dev)
    stream = torch.cuda.Stream(device=dev)
    stream.wait_stream(torch.cuda.current_stream())
    it = [0]

    def step():
        i = it[0]
        phi_stack(pairs, stacks[i & 1], reset, out=stacks[(i + 1) & 1], stream=stream)
        it[0] = i + 1

    with torch.cuda.stream(stream):
        for _ in range(a.warmup):
            step()
    stream.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0.record(stream)
        for _ in range(a.steps):
            step()
        ev1.record(stream)
    stream.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    us = 1e3 * ev0.elapsed_time(ev1) / a.steps
    if dist.is_initialized():
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        work = n * PHI_STACK_BYTES_PER_PAIR
        ach = work / (us * 1e-6) / 1e9
        traffic = measured_traffic(n, 0, "phi", "phi_stack_kernel")
        out = {"metric": "env-steps/sec (phi+forward+sample+update) at 1/2/4/8 MI355X; % roofline",
               "value": round(n * world * a.steps / elapsed, 1), "unit": "frame pairs/s (phi stage only)",
               "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": round(1e3 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "u8", "data": "synthetic uniform RGB 210x160 frame pairs",
               "config": {"workload": "c5: dqn_phi stress, %d frame pairs/batch 210x160 RGB -> 84x84x4 uint8" % n,
                          "pairs_per_gpu": n, "parallelism": "dp%d" % world},
               "roofline": {"bound": "hbm", "kernel": "phi_stack_kernel", "achieved": round(ach, 1),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                            "traffic": traffic, "avg_launch_us": round(us, 2), "work_per_launch": work,
                            "peak_measured": copy_peak["GB/s"] if copy_peak else None,
                            "frac_measured_peak": round(ach / copy_peak["GB/s"], 4) if copy_peak else None},
               "hbm_copy_peak": copy_peak,
               "cpu_baseline": None}
        print(json.dumps(out))
    if dist.is_initialized():
        dist.destroy_process_group()


def secondary_line(a, pkg, dev, workload):
    """One more BASELINE workload on this GPU (N = 1), measured as the headline
    is: W warmup windows, K timed windows between two synchronizes (wall
    clock), then 100 windows between HIP events for the median.  The window is
    the library default's: env-group chains as one graph replay from 1,024
    envs (C3), eager launches for one chain."""
    w_arch, N, A = WORKLOADS[workload]
    T, P = a.t_max, a.pool
    Model = pkg.A3CLSTM if w_arch == "lstm" else pkg.A3CFF
    model = Model(A, n_envs=N, t_max=T, seed=1234, init_seed=0, device=dev, frames="pairs")
    opt = pkg.RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(pkg.GradientClipping(40))
    opt.anneal_total_steps, opt.n_total_envs = 8 * 10 ** 7, N
    agent = pkg.A3C(model, opt, T, 0.99, beta=1e-2, collectives=False)
    pairs, rewards, dones = synth_pools(N, P, 0, dev)
    groups = len(model.net.env_groups(model.net.default_env_groups()))
    stream = torch.cuda.Stream(device=dev)
    stream.wait_stream(torch.cuda.current_stream())
    graph = None
    with torch.cuda.stream(stream):
        agent.run_window(pairs, rewards, dones, P, first=True, stream=stream)
        if groups > 1:   # captured before the warmup windows, which then run right before the timed ones
            agent.run_window(pairs, rewards, dones, P, stream=stream)   # (creates the side streams)
            stream.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                agent.run_window(pairs, rewards, dones, P, stream=stream)

    def window():
        if graph is not None:
            graph.replay()
        else:
            agent.run_window(pairs, rewards, dones, P, stream=stream)

    with torch.cuda.stream(stream):
        for _ in range(max(0, a.warmup - 1)):
            window()
    stream.synchronize()

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(a.steps):
            window()
    stream.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    M = 100
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(M + 1)]
    with torch.cuda.stream(stream):
        evs[0].record(stream)
        for i in range(M):
            window()
            evs[i + 1].record(stream)
    stream.synchronize()
    med = float(np.median([evs[i].elapsed_time(evs[i + 1]) for i in range(M)]))
    out = {"workload": "%s: A3C %s NIPS-DQN head, %d envs x t_max=%d on one GPU, A = %d" % (workload, w_arch.upper(),
                                                                                           N, T, A),
           "value": round(N * T * a.steps / elapsed, 1), "unit": "env-steps/s", "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 4), "env_groups": groups,
           "graph": graph is not None, "median_window_ms": round(med, 4),
           "median_env_steps_per_s": round(N * T / (med * 1e-3), 1),
           "params_finite": bool(torch.isfinite(model.net.params).all())}
    del graph, agent, opt, model, pairs, rewards, dones
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def timed_region_diag(a, window, stream):
    """The timed region's shape again (synchronize, K windows, synchronize),
    a.timed_diag times, with a HIP event recorded before the first window and
    after each one: per repetition the host-timed mean, the event-timed
    windows (first one apart), and the host time outside the events (launch
    of the first kernel, the final synchronize).  Half the repetitions start
    after a 20 ms idle sleep (a clock ramp would show in their first windows)."""
    reps = []
    for r in range(a.timed_diag):
        if r % 2 == 1:
            time.sleep(0.02)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            evs[0].record(stream)
            for i in range(a.steps):
                window()
                evs[i + 1].record(stream)
        stream.synchronize()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)]
        reps.append({"idle_before_ms": 20 if r % 2 == 1 else 0, "host_mean_ms": round(1e3 * el / a.steps, 4),
                     "event_mean_ms": round(float(np.mean(ms)), 4), "first_ms": round(ms[0], 4),
                     "second_ms": round(ms[1], 4) if len(ms) > 1 else None,
                     "rest_median_ms": round(float(np.median(ms[1:])), 4) if len(ms) > 1 else None,
                     "outside_events_ms": round(1e3 * el - float(np.sum(ms)), 4)})
    return reps


def main(a):
    mp_ctx = None
    if a.cpu_seconds > 0 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # CPU baseline leg (ii) workers are forked by a forkserver started
        # here, before anything touches the GPU (no worker is a fork of a GPU
        # process); it preloads the oracle's CPU baseline module
        import multiprocessing as mp
        from multiprocessing import forkserver
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        mp_ctx = mp.get_context("forkserver")
        mp_ctx.set_forkserver_preload(["cpu_baseline"])
        forkserver.ensure_running()
    world, rank, local, collectives = init_dist(a.dist_timeout)
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}")
    dev = torch.device("cuda", local)
    seen = ranks_seen(dev)
    if collectives and seen != world:
        raise SystemExit(f"bench.py: {seen} ranks answered the all-reduce, expected {world}")
    pkg = _import_pkg()
    A3C, RMSpropAsync, GradientClipping = pkg.A3C, pkg.RMSpropAsync, pkg.GradientClipping
    from asyncrl_amd._lib import LEARN_CONV
    copy_peak = measure_copy_peak(dev) if (rank == 0 and a.copy_peak) else None
    w_arch, w_envs, w_A = WORKLOADS[a.workload]
    if w_arch == "phi":
        return bench_phi(a, world, rank, dev, w_envs, copy_peak)
    arch = a.arch or w_arch
    A = a.actions or (w_A if arch == w_arch else (6 if arch == "lstm" else 4))
    N, T = a.envs_per_gpu or w_envs, a.t_max
    Model = {"ff": pkg.A3CFF, "lstm": pkg.A3CLSTM, "nature": pkg.A3CFFNature, "doom_ff": pkg.DoomA3CFF,
             "doom_lstm": pkg.DoomA3CLSTM}[arch]
    nat = arch == "nature"
    lstm = arch in ("lstm", "doom_lstm")
    doom = arch.startswith("doom")
    if doom and not a.actions:
        A = 3                                          # train_a3c_doom.py:105
    conv_fwd_flop = NAT_CONV_FWD_FLOP_PER_ENV if nat else DOOM_CONV_FWD_FLOP_PER_ENV if doom else CONV_FWD_FLOP_PER_ENV
    fc_fwd_flop = NAT_FC_FWD_FLOP_PER_ENV if nat else FC_FWD_FLOP_PER_ENV
    conv_bwd_flop = NAT_CONV_BWD_FLOP_PER_SAMPLE if nat else DOOM_CONV_BWD_FLOP_PER_SAMPLE if doom else \
        CONV_BWD_FLOP_PER_SAMPLE
    hid_bytes = 2 * HID_BYTES if nat else HID_BYTES
    model = Model(A, n_envs=N, t_max=T, seed=1234, env_offset=rank * N, init_seed=0, device=dev, frames="pairs")
    opt = RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(GradientClipping(40))
    opt.anneal_total_steps = 8 * 10 ** 7        # a3c_ale.py:200 --steps default
    opt.n_total_envs = N * world
    agent = A3C(model, opt, T, 0.99, beta=1e-2, collectives=collectives)
    if doom:
        dH, dW = a.doom_width * 3 // 4, a.doom_width
        pairs, rewards, dones = synth_rgb_pools(N, a.pool, rank, dev, dH, dW)
        phi_bytes = rgb_phi_bytes(dH, dW)
    else:
        pairs, rewards, dones = synth_pools(N, a.pool, rank, dev)
        phi_bytes = PHI_BYTES_PER_ENV_STEP
    P = a.pool

    n_groups = len(model.net.env_groups(a.env_groups or model.net.default_env_groups()))
    use_graph = False if a.no_graph else a.graph == "on" or (a.graph == "auto" and n_groups > 1)
    graph = conv_graph = None
    stream = torch.cuda.Stream(device=dev)
    stream.wait_stream(torch.cuda.current_stream())

    def window():
        if graph is not None:
            graph.replay()
            if collectives:
                agent.finish_window(stream=stream, conv=conv_graph.replay if conv_graph is not None else None)
            else:
                agent.t += T
        else:
            agent.run_window(pairs, rewards, dones, P, first=False, stream=stream, env_groups=(a.env_groups or None))

    with torch.cuda.stream(stream):
        agent.run_window(pairs, rewards, dones, P, first=True, stream=stream, env_groups=(a.env_groups or None))
        for _ in range(max(0, a.warmup - 1)):
            agent.run_window(pairs, rewards, dones, P, stream=stream, env_groups=(a.env_groups or None))
        if use_graph:
            stream.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                # one window; with >1 rank the all-reduce + optimizer stay eager, and with the
                # overlapped all-reduce the conv backward is a second graph replayed while the
                # FC / heads section of the gradient is on the wire (A3C._reduce_and_step)
                agent.run_window(pairs, rewards, dones, P, stream=stream, split_update=collectives,
                                 env_groups=(a.env_groups or None))
            if collectives and agent._overlap_allreduce():
                cg = torch.cuda.CUDAGraph()
                with torch.cuda.graph(cg, stream=stream):
                    model.net.learn_parts([LEARN_CONV], agent.gamma, agent.beta, agent._vcoef,
                                          agent.clip_reward, stream=stream)
                conv_graph = cg
            graph = g
            agent.t -= 0 if collectives else T
            for _ in range(2):
                window()
    stream.synchronize()

    # ---------------------------------------------------------------- timed region
    if collectives:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(a.steps):
            window()
    t_enq = time.perf_counter() - t0      # host time to issue the K windows (eager launches / replays)
    stream.synchronize()
    if collectives:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if collectives:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    units = N * T * world * a.steps
    value = units / elapsed
    ms_step = 1e3 * elapsed / a.steps

    diag = timed_region_diag(a, window, stream) if a.timed_diag > 0 else None

    # per-window distribution (median over >= 100 windows): more
    # windows after the timed region, each between two HIP events on the bench
    # stream (which every part of a window, collectives included, joins)
    windows = None
    if a.median_windows > 0:
        M = a.median_windows
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(M + 1)]
        with torch.cuda.stream(stream):
            evs[0].record(stream)
            for i in range(M):
                window()
                evs[i + 1].record(stream)
        stream.synchronize()
        ms = np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(M)])
        q = np.percentile(ms, [10, 50, 90])
        med = float(q[1])
        if collectives:
            t = torch.tensor([med], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            med = float(t.item())
        windows = {"n": M, "median_ms": round(med, 4), "p10_ms": round(float(q[0]), 4),
                   "p90_ms": round(float(q[2]), 4), "median_env_steps_per_s": round(N * T * world / (med * 1e-3), 1),
                   "note": "HIP events per window on the bench stream; median = max over ranks of each rank's "
                           "median, p10 / p90 rank 0's"}
    finite = bool(torch.isfinite(model.net.params).all())
    replicas = None
    if collectives:   # every rank applied the same update to the same reduced gradient (distributed.py)
        from asyncrl_amd.distributed import replicas_identical
        replicas = bool(replicas_identical(model.net.params) and replicas_identical(model.net.ms))

    # ---------------------------------------------------------------- window timeline
    # More eager windows with a HIP event recorded after every stage launch
    # (arl_stamps_*; A3C adds one after each collective): consecutive
    # intervals split a window into its stages as it ran, launch boundaries
    # included, so the per-stage shares add up to the window.  Every rank runs
    # them (the collectives need all ranks); rank 0 reports its own.
    timeline = None
    net = model.net
    if a.stamp_windows > 0 and not use_graph and n_groups == 1 and not nat:
        from asyncrl_amd._lib import STAGE_NAMES

        def stamped(n_win, period=0):
            net.stamps_begin(n_win * 64 + 8)
            if period:
                net.stamps_sparse(period)
            with torch.cuda.stream(stream):
                if not period:
                    net.stamp(16, stream=stream)   # the mark the first interval starts from (ARL_STAGE_OTHER)
                for _ in range(n_win):
                    window()
            stream.synchronize()
            ms_st, names = net.stamps_end()
            return ms_st[1:], ["allreduce_wait" if x == STAGE_NAMES[15] else x for x in names[1:]]

        # dense: every stage launch stamped (each event lengthens the interval it closes by ~1 us);
        # sparse: n_st stamp calls a window, window w records only calls t - 1 and t (t = w mod n_st),
        # so each launch's in-window interval is timed with no other event in its window
        m_dense = min(a.stamp_windows, 20)
        ms_d, names_d = stamped(m_dense)
        n_st = len(ms_d) // m_dense
        dense_ms = float(ms_d.sum()) / m_dense
        reps = max(4, -(-a.stamp_windows // n_st))
        ms_s, names_s = stamped(n_st * reps, n_st)
        per = {}
        for x, name in zip(ms_s, names_s):
            if x >= 0:
                per.setdefault(name, []).append(float(x))
        count = {}
        for name in names_d[:n_st]:
            count[name] = count.get(name, 0) + 1
        stages = {k: {"window_share_us": round(1e3 * float(np.mean(per[k])) * count[k], 2),
                      "launches_per_window": count[k], "us_per_launch": round(1e3 * float(np.mean(per[k])), 3),
                      "samples": len(per[k])} for k in count if k in per}
        total_ms = sum(v["window_share_us"] for v in stages.values()) / 1e3
        timeline = {"windows": n_st * reps, "stamps_per_window": n_st, "sum_of_shares_ms": round(total_ms, 4),
                    "stages": stages, "dense_windows": m_dense, "dense_mean_window_ms": round(dense_ms, 4),
                    "note": "sparse stamps (arl_stamps_sparse): each stage launch's interval from the previous "
                            "launch's event to its own, timed in windows that record only those two events, so "
                            "a launch's share includes its dependent-launch boundary; dense_mean_window_ms = "
                            "windows with every launch stamped; allreduce_wait = the compute stream's wait for "
                            "the collectives (A3C._reduce_and_step)"}
        if windows is not None:
            timeline["unstamped_median_ms"] = windows["median_ms"]
            # the raw sparse sum is the checked quantity (tests/test_gpu_bench.py: <= 1.08 x the unstamped
            # median at C4): each interval carries one event's cost beyond the launch it times
            timeline["sum_vs_unstamped_median"] = round(total_ms / windows["median_ms"], 4)
            timeline["dense_vs_unstamped_median"] = round(dense_ms / windows["median_ms"], 4)
            # A labelled ESTIMATE, not used for any assertion or rate: the cost of one event, measured
            # independently from the dense windows (every launch stamped) against the unstamped median,
            # taken off each sparse interval.  corrected_sum_vs_unstamped_median is then a real check of
            # that estimate (nothing forces it to 1).
            x_ms = max(0.0, (dense_ms - windows["median_ms"]) / n_st)
            timeline["estimated_event_cost_us"] = round(1e3 * x_ms, 3)
            for v in stages.values():
                v["us_per_launch_est_eventfree"] = round(v["us_per_launch"] - 1e3 * x_ms, 3)
            timeline["corrected_sum_vs_unstamped_median"] = round(
                (total_ms - x_ms * n_st) / windows["median_ms"], 4)

    # ---------------------------------------------------------------- per-kernel roofline
    # Each stage's algorithmic work per launch over its
    # in-window time per launch (the timeline above); every stage is also
    # re-launched alone kernel-reps times back to back between two HIP events
    # on the bench stream ("standalone_us", beside it).  The stage with the
    # largest in-window share is the "roofline" kernel.
    roof, kernels = None, None
    if rank == 0:
        S = N * T

        def timed(fn):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for i in range(3):
                fn(i)
            ev0.record(stream)
            for i in range(a.kernel_reps):
                fn(i)
            ev1.record(stream)
            ev1.synchronize()
            return 1e3 * ev0.elapsed_time(ev1) / a.kernel_reps

        specs = [  # name, kernel, launch fn, nominal launches per window, bound, algorithmic work per launch
            # a window observes steps 1..T (step 0 of a window is the previous window's bootstrap observation)
            ("phi", "rgb_ring_kernel" if doom else "phi_ring_kernel",
             lambda i: net.observe(1 + i % T, pairs, rewards, dones, P, stream=stream), T, "hbm",
             N * phi_bytes),
            ("conv_fwd", "gemm_kernel x3 (implicit-GEMM convs)" if nat else
             f"conv_fwd_kernel<{conv_epw(N)}>",
             lambda i: net.run_stage("conv_fwd", i % T, stream=stream), T + 1, "mfma",
             N * conv_fwd_flop),
            ("fc_fwd", "gemm_kernel + reduce_grad_kernel" if nat else
             ("fc_fwd_big_kernel" if fc_big(N) else "fc_fwd_kernel") +
             (" (split-K partials)" if (not lstm or lstm_xred(N)) else " (+ ticket reduce)"),
             lambda i: net.run_stage("fc_fwd", i % T, stream=stream), T + 1, "mfma", N * fc_fwd_flop),
            # FF NIPS / Doom FF: the FC split-K reduce + bias + relu runs in the policy launch
            # (policy_fc_kernel): it also reads the 8 partial slabs and writes h
            ("policy", "policy_kernel" if (nat or lstm) else "policy_fc_kernel (FC reduce + heads)",
             lambda i: net.run_stage("policy", i % T, stream=stream), T + 1, "hbm",
             N * (hid_bytes + 12 * A + 12) + (0 if (nat or lstm) else N * (FC_SPLIT + 1) * hid_bytes)),
            ("fc_bwd", "gemm_kernel x2 + reduce_grad_kernel" if nat else "fc_bwd_kernel (dW + da2 + heads dW)",
             lambda i: net.run_stage("fc_bwd", 0, stream=stream), 1, "mfma", 2 * fc_fwd_flop * S),
            ("conv_bwd", "gemm_kernel x9 + reduce_grad_kernel x3" if nat else
             ("conv_bwd_kernel" if os.environ.get("ARL_CB_WS", "") == "0" else "conv_bwd_ws_kernel"),
             lambda i: net.run_stage("conv_bwd", 0, stream=stream), 1, "mfma", S * conv_bwd_flop),
            # LSTM: the gate kernel (LSTM_XRED: it also forms x from the FC's partials), the
            # truncated-BPTT steps, the gate weight gradients + dfc (a3c_ale.py:50-51,62)
            ("lstm_gates", "lstm_gates_kernel" + ("<true> (FC reduce + gates + cell)" if lstm_xred(N) else "<false>"),
             lambda i: net.run_stage("lstm_gates", i % T, stream=stream), T + 1, "mfma",
             N * LSTM_GATES_FLOP_PER_ENV) if lstm and not doom else None,
            ("lstm_bptt", "lstm_bptt_kernel (dh GEMM + cell backward)",
             lambda i: net.run_stage("lstm_bptt", T - 1 - i % (T - 1), stream=stream), T - 1, "mfma",
             N * LSTM_BPTT_FLOP_PER_ENV) if lstm and not doom and T > 1 else None,
            ("lstm_wgrad", "fc_bwd_kernel<ShapeLSTM> (gate dW / db + dfc, straight into the gradient)",
             lambda i: net.run_stage("lstm_wgrad", stream=stream), 1, "mfma",
             S * LSTM_WGRAD_FLOP_PER_SAMPLE) if lstm and not doom else None,
            # the update kernel as the window runs it: clip 40 from the norm the learner left (lr 0 alone)
            ("rmsprop", "rmsprop_kernel (clip + RMSProp + window advance)",
             (lambda i: net.run_stage("rmsprop", stream=stream)) if not nat else
             (lambda i: net.optimize(lr0=0.0, clip=0.0, stream=stream)), 1, "hbm",
             net.n_params * RMSPROP_BYTES_PER_PARAM),
            # the learner's small HBM-bound launches (NIPS heads): returns + loss gradient + heads dh,
            # the conv backward's slab reduce, the gradient's squared norm (GradientClipping)
            None if nat else
            # (FF one-call windows: folded into the bootstrap step's policy launch, policy_fc_returns_kernel)
            ("returns", "returns_heads_kernel", lambda i: net.run_stage("returns", stream=stream), 1, "hbm",
             returns_bytes(N, T, A, mask=not lstm)),
            None if nat else
            ("conv_reduce", "reduce_conv_bwd_kernel" + (" (+ clip norm)" if not collectives else ""),
             lambda i: net.run_stage("conv_reduce", stream=stream), 1, "hbm",
             (conv_bwd_blocks(S) + 1) * CONV_SLAB_FLOATS * 4 + (net.n_params * 4 if not collectives else 0)),
            # with one rank the clip norm is folded into the conv reduce (A3C: arl_net_set_norm_fold), so
            # the grad_sqnorm launch is not in the window; its time is listed for reference
            None if nat else
            ("grad_sqnorm", "grad_sqnorm_kernel", lambda i: net.run_stage("grad_sqnorm", stream=stream),
             0 if not collectives else 1, "hbm", net.n_params * 4),
        ]
        tl = timeline["stages"] if timeline is not None else {}
        kernels = {}
        with torch.cuda.stream(stream):
            for name, kname, fn, calls, bound, work in filter(None, specs):
                # the update stage runs with lr 0 (p unchanged) but still rewrites the RMSProp statistics:
                # time it on the live buffers, then put ms back (the line's params_finite / replica checks and
                # any later window see the state the timed windows left)
                ms_keep = net.ms.clone() if name == "rmsprop" else None
                us_alone = timed(fn)
                if ms_keep is not None:
                    stream.synchronize()
                    net.ms.copy_(ms_keep)
                win = tl.get(name)
                if win is None and timeline is not None:
                    calls = 0   # not in the window (FF: the returns run in the bootstrap policy launch)
                # the raw in-window interval (one event's cost included: a lower bound on the kernel's rate)
                us = win["us_per_launch"] if win is not None else us_alone
                cyc = mfma_cycles(name, N, T, arch) if (bound == "mfma" and arch in ("ff", "lstm")) else None
                ideal = None if cyc is None else mfma_ideal_cycles(name, N, T)
                if bound == "hbm":
                    peak, unit = HBM_PEAK_GBS, "GB/s"
                    rate = lambda t_us: work / (t_us * 1e-6) / 1e9   # noqa: E731
                elif ideal is not None:
                    # the f32-equivalent ceiling of the instructions this kernel runs its contractions on
                    peak, unit = round(work / (ideal / (SIMDS * CLK_HZ)) / 1e12, 1), "TFLOP/s"
                    rate = lambda t_us: work / (t_us * 1e-6) / 1e12   # noqa: E731
                else:   # exact f32 generic GEMMs (Nature head)
                    peak, unit = F32_MFMA_PEAK_TFS, "TFLOP/s"
                    rate = lambda t_us: work / (t_us * 1e-6) / 1e12   # noqa: E731
                ach, ach1 = rate(us), rate(us_alone)
                kernels[name] = {"kernel": kname, "bound": bound, "avg_launch_us": round(us, 2),
                                 "time_source": "window" if win is not None else "standalone",
                                 "launches_per_window": win["launches_per_window"] if win is not None else calls,
                                 "window_share_us": win["window_share_us"] if win is not None else round(us * calls, 1),
                                 "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                                 ("bytes" if bound == "hbm" else "flop") + "_per_launch": int(work),
                                 "standalone_us": round(us_alone, 2), "standalone_frac": round(ach1 / peak, 4)}
                if cyc is not None:
                    kernels[name]["issued"] = {
                        "mfma_cycles_per_launch": int(cyc),
                        "frac_issued": round(cyc / (SIMDS * CLK_HZ * us * 1e-6), 4),
                        "standalone_frac_issued": round(cyc / (SIMDS * CLK_HZ * us_alone * 1e-6), 4),
                        "padding": round(cyc / ideal, 4)}
        for tname, win in tl.items():   # timeline stages without a standalone form (LSTM cells, collectives)
            if tname not in kernels:
                kernels[tname] = {"kernel": tname, "bound": None, "time_source": "window",
                                  "avg_launch_us": win["us_per_launch"],
                                  "launches_per_window": win["launches_per_window"],
                                  "window_share_us": win["window_share_us"]}
        dom = max((k for k in kernels if kernels[k]["bound"] is not None), key=lambda k: kernels[k]["window_share_us"])
        d = kernels[dom]
        traffic = measured_traffic(N, T, arch, d["kernel"].split(" (")[0])
        roof = {"bound": d["bound"], "kernel": d["kernel"], "achieved": d["achieved"], "peak": d["peak"],
                "unit": d["unit"], "frac": d["frac"], "traffic": traffic, "avg_launch_us": d["avg_launch_us"],
                "time_source": d["time_source"], "standalone_us": d["standalone_us"],
                "standalone_frac": d["standalone_frac"],
                "work_per_launch": d.get("flop_per_launch", d.get("bytes_per_launch")),
                "peak_note": (("exact f32 MFMA (v_mfma_f32_16x16x4_f32) vs the dense fp32 matrix peak" if nat else
                               "achieved = algorithmic f32 FLOPs / time; peak = the f32-equivalent ceiling of the "
                               "instructions the kernel issues (bf16 v_mfma_f32_16x16x32 at the 2.5 PFLOP/s dense "
                               "bf16 peak / 3 or 6 exact-split terms per f32 product, exact f32 v_mfma_f32_16x16x4 "
                               "at 157.3); frac_issued = the MFMA cycles it issues (padding included) / the "
                               "chip's matrix-pipe cycles in that time, the model of SQ_VALU_MFMA_BUSY")
                              if d["bound"] == "mfma" else "HBM3E spec peak") +
                             ("; time = the raw in-window interval per launch (sparse window timeline), one "
                              "timing event and the launch boundary included: a lower bound on the kernel's rate"
                              if d["time_source"] == "window" else "")}
        if "issued" in d:
            roof["frac_issued"] = d["issued"]["frac_issued"]
            roof["mfma_cycles_per_launch"] = d["issued"]["mfma_cycles_per_launch"]
        if copy_peak is not None:
            # HBM-bound stages also against the copy rate measured on this GPU
            for k in kernels.values():
                if k["bound"] == "hbm":
                    k["frac_measured_peak"] = round(k["achieved"] / copy_peak["GB/s"], 4)
            if roof["bound"] == "hbm":
                roof["peak_measured"] = copy_peak["GB/s"]
                roof["frac_measured_peak"] = round(roof["achieved"] / copy_peak["GB/s"], 4)
        if "phi" in kernels and not doom:
            # phi on the bytes it moves: the 168 of 210 source rows the resize taps touch (x2 frames x
            # 480 B) + the plane written, besides SURVEY 8(d)'s whole-pair basis
            k = kernels["phi"]
            moved = N * (PHI_TAP_ROWS * 160 * 3 * 2 + PLANE_BYTES)
            ach = moved / (k["avg_launch_us"] * 1e-6) / 1e9
            k["moved_basis"] = {"bytes_per_launch": moved, "achieved": round(ach, 2), "unit": "GB/s",
                                "frac": round(ach / HBM_PEAK_GBS, 4)}
            if copy_peak is not None:
                k["moved_basis"]["frac_measured_peak"] = round(ach / copy_peak["GB/s"], 4)

    cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0 and arch == "ff":
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_baseline  # noqa: E402  (oracle/, CPU baseline leg only)
        cpu = cpu_baseline.run(seconds=a.cpu_seconds, t_max=T, n_actions=4)        # leg (i): 1 process, 1 core
        cpu["cpu_model"] = cpu_baseline.cpu_model()
        # leg (ii) as BASELINE.md §2 states it: P = physical cores, one process each (async.py:68-90);
        # on a box whose cgroup quota grants fewer CPUs they time-share them, so the quota-sized run
        # (P = CPUs this process may use) is recorded beside it
        phys, _, avail = cpu_baseline.host_cores()
        par = cpu_baseline.run_parallel(seconds=a.cpu_seconds, t_max=T, n_actions=4, procs=phys, ctx=mp_ctx)
        if avail < phys:
            par["quota_sized"] = cpu_baseline.run_parallel(seconds=a.cpu_seconds, t_max=T, n_actions=4, ctx=mp_ctx)
        cpu["parallel"] = par
        cpu["gpu_vs_parallel"] = round(value / par["value"], 1)

    secondary = None
    sec = a.secondary if a.secondary != "auto" else ("c3" if (a.workload == "c4" and world == 1 and arch == "ff")
                                                    else "none")
    if world == 1 and sec not in ("", "none"):   # (the headline's buffers stay: 288 GB of HBM)
        secondary = [secondary_line(a, pkg, dev, w.strip()) for w in sec.split(",") if w.strip()]

    if rank == 0:
        out = {
            "metric": "env-steps/sec (phi+forward+sample+update) at 1/2/4/8 MI355X; % roofline",
            "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": ("synthetic (uniform RGB24 %dx%d ViZDoom-shaped screens" % (dH, dW) if doom else
                     "synthetic (uniform RGB 210x160 frame pairs") + ", rewards P(!=0)=0.05, terminals p=1/500)",
            "config": {"workload": ("%s: A3C %s " + ("Nature" if nat else "NIPS (RGB)" if doom else "NIPS") + "-DQN head, %d envs x t_max=%d per GPU (phi + conv head + sampling "
                                    "+ n-step returns + backward + clip + RMSProp)") % (a.workload, arch.upper(), N, T),
                       "envs_per_gpu": N, "global_envs": N * world, "t_max": T, "n_actions": A, "arch": arch,
                       "graph": use_graph, "env_groups": len(model.net.env_groups(a.env_groups or model.net.default_env_groups())),
                       "parallelism": "dp%d" % world,
                       "units_per_step": N * T * world},
            "host_issue_ms_per_step": round(1e3 * t_enq / a.steps, 4),
            "ranks_seen": seen, "collectives": (("rccl" if dist.get_backend() == "nccl" else dist.get_backend())
                                                if collectives else None),
            "allreduce_bytes_per_window": (4 * model.net.grads.numel()) if collectives else 0,
            "replicas_identical": replicas,
            "windows": windows, "timeline": timeline, "hbm_copy_peak": copy_peak,
            **({"timed_region_diag": diag} if diag is not None else {}),
            "roofline": roof, "kernels": kernels, "cpu_baseline": cpu, "params_finite": finite,
            "secondary": secondary,
        }
        print(json.dumps(out), flush=True)
    if collectives:
        dist.destroy_process_group()


if __name__ == "__main__":
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    main(args)
