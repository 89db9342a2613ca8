"""Worker for tests/test_gpu_dist.py::test_two_rank_window_matches_oracle: the
N > 1 learner window the 8-GPU bench runs, checked against the oracle.

Two ranks share the one GPU of the box (gloo transport: RCCL needs one GPU per
rank), each owning 256 envs (BASELINE configs[3]'s leg is 512; 256 keeps the
CPU oracle at tens of seconds).  Every rank runs exactly the bench's window:
A3C(collectives=True by world size) -> run_window on a side stream, eager:
T x (phi, forward, sample), bootstrap, returns, FC backward, the FC / heads
section of the gradient all-reduced while the conv backward runs, the conv
section all-reduced, then GradientClipping(40) from grad_sqnorm on the REDUCED
gradient and RMSProp (a3c.py:129-143, async.py:68-90: the reference's
per-process update, here on the sum over both ranks' envs).

Per window (two windows, the second from the first's updated parameters and
RMSProp statistics) the optimizer's entry is intercepted to snapshot the
reduced gradient, parameters and ms exactly as RMSProp sees them.  Each rank
computes its shard's oracle gradient (f64, per env chunk, oracle.ff_window_grads)
and writes it to the run directory; rank 0 sums both shards in f64 and checks
  * the all-reduced gradient vs the oracle sum: every tensor norm-scaled at
    1e-5 and componentwise at 1e-5 of each element's own error scale;
  * the clip: oracle norm (f64) > 40 so clipping is active, and the device's
    f64 norm of what it reduced within 1e-5 of the oracle's;
  * the update: post-RMSProp parameters / ms vs oracle.rmsprop_update on the
    snapshot with the oracle-rate clip (1e-6, the same gradient) and on the
    oracle's summed gradient (1e-5, norm-scaled on the parameter change);
and both ranks check that params, ms and the reduced gradient are bitwise
identical across ranks.  Results: <outdir>/res.json."""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "async-rl_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

from datetime import timedelta  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle as O  # noqa: E402
from conftest import close_grad, close_normscaled  # noqa: E402
from sim import OracleEnvView, make_pools, oracle_window_chunks  # noqa: E402

N_LOCAL = int(os.environ.get("ARL_DIST_ENVS", "256"))
T, P, A, CLIP, LR = 5, 6, 4, 40.0, 7e-4
RTOL = 1e-5


def main():
    outdir = sys.argv[1]
    dist.init_process_group("gloo", timeout=timedelta(seconds=240))
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    gpu = torch.device("cuda:0")
    from asyncrl_amd import A3C, A3CFF, GradientClipping, RMSpropAsync
    from asyncrl_amd.distributed import replica_checksum, replicas_identical

    rng = np.random.default_rng(100 + rank)          # each rank its own envs
    pairs, rewards, dones = make_pools(rng, P, N_LOCAL, "uniform", p_done=0.1)
    model = A3CFF(A, n_envs=N_LOCAL, t_max=T, seed=77, env_offset=rank * N_LOCAL, init_seed=5, frames="pairs",
                  device=gpu)
    opt = RMSpropAsync(lr=LR, eps=0.1, alpha=0.99).setup(model)
    opt.add_hook(GradientClipping(CLIP))
    agent = A3C(model, opt, T, 0.99)
    net = model.net
    assert agent.collectives and agent._overlap_allreduce(), "not the sectioned N > 1 window"

    snap = {}
    update = opt.update

    def intercepted(*a, **kw):            # runs on the window's stream (A3C._reduce_and_step)
        snap["g"], snap["p"], snap["ms"] = net.grads.clone(), net.params.clone(), net.ms.clone()
        return update(*a, **kw)

    opt.update = intercepted
    view = OracleEnvView(pairs, dones)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(gpu)  # noqa: E731
    dp, dr, dd = dev(pairs), dev(rewards), dev(dones)
    stream = torch.cuda.Stream(device=gpu)
    stream.wait_stream(torch.cuda.current_stream())
    res = {"rank": rank, "world": world, "envs_per_rank": N_LOCAL, "windows": []}
    names = list(net.layout)
    for w in range(2):
        params = net.state_dict()
        with torch.cuda.stream(stream):
            agent.run_window(dp, dr, dd, P, first=(w == 0), stream=stream)
        stream.synchronize()
        # this rank's shard of the oracle gradient at the window's parameters
        k0 = w * T
        states, boot = view.states_f32(k0, T)
        r, d = view.window_rd(rewards, k0, T)
        acts = net.buffer("actions", torch.int32, (T + 1, N_LOCAL))[:T].cpu().numpy()
        acts_dev = (net.buffer("a1", torch.float32, (T + 1, N_LOCAL, 16, 20, 20))[:T].cpu().numpy(),
                    net.buffer("a2", torch.float32, (T + 1, N_LOCAL, 32, 9, 9))[:T].cpu().numpy(),
                    net.buffer("hfc", torch.float32, (T + 1, N_LOCAL, 256))[:T].cpu().numpy())
        for t in range(T):   # the shard's own draws: Philox keyed by global env id
            probs = net.buffer("probs", torch.float32, (T + 1, N_LOCAL, A))[t].cpu().numpy()
            u = O.sample_uniforms(77, np.arange(rank * N_LOCAL, (rank + 1) * N_LOCAL, dtype=np.uint64), k0 + t)
            assert (O.sample_from_uniform(probs, u) == acts[t]).all(), (rank, w, t)
        g, aux = oracle_window_chunks(O.ARCH_FF, params, states, acts, r, d, boot, acts_dev=acts_dev, return_f64=True)
        np.savez(os.path.join(outdir, f"shard{rank}_w{w}.npz"),
                 **{"g|" + k: v for k, v in g.items()},
                 **{"m2|" + k: v.astype(np.float64) ** 2 for k, v in aux["grad_mag"].items()})
        same = {k: replicas_identical(snap[k]) for k in ("g", "p", "ms")}
        same["params_after"] = replicas_identical(net.params)
        same["ms_after"] = replicas_identical(net.ms)
        dist.barrier()
        win = {"w": w, "identical": same, "checksum_params": replica_checksum(net.params)}
        if rank == 0:
            gsum, m2 = {}, {}
            for r_ in range(world):
                with np.load(os.path.join(outdir, f"shard{r_}_w{w}.npz")) as z:
                    for key in z.files:
                        kind, k = key.split("|", 1)
                        tgt = gsum if kind == "g" else m2
                        tgt[k] = tgt.get(k, 0.0) + z[key]
            got = net.state_dict(snap["g"])
            bad = []
            for k in names:
                ok, e_ns = close_normscaled(got[k], gsum[k], RTOL)
                ok2, e_el = close_grad(got[k], gsum[k], np.sqrt(m2[k]), RTOL)
                win.setdefault("grad_err_normscaled", {})[k] = e_ns
                win.setdefault("grad_err_componentwise", {})[k] = e_el
                if not (ok and ok2):
                    bad.append(k)
            win["grad_bad"] = bad
            # the clip: GradientClipping(40) over the whole reduced gradient
            norm_o = math.sqrt(sum(float((v ** 2).sum()) for v in gsum.values()))
            gd = snap["g"].double()
            norm_d = float(gd.pow(2).sum().sqrt())
            win["norm_oracle"], win["norm_device"] = norm_o, norm_d
            win["norm_rel_err"] = abs(norm_d - norm_o) / norm_o
            win["clip_active"] = norm_o > CLIP
            # the update: RMSProp on the snapshot (the exact gradient the kernel saw), clip rate from
            # the oracle's f64 norm of that gradient, and on the oracle's own summed gradient
            p0, ms0 = snap["p"].cpu().numpy(), snap["ms"].cpu().numpy()
            g0 = snap["g"].cpu().numpy()
            (gc,), _ = O.clip_grads([g0], CLIP, exact_norm=True)
            p1, m1 = O.rmsprop_update(p0, ms0, gc, LR)
            pa, ma = net.params.cpu().numpy(), net.ms.cpu().numpy()
            win["update_err_same_grad"] = [close_normscaled(pa - p0, p1 - p0, 1e-6)[1],
                                           close_normscaled(ma, m1, 1e-6)[1]]
            flat_o = np.zeros_like(g0, dtype=np.float64)
            for k in names:
                off, shape = net.layout[k]
                flat_o[off:off + int(np.prod(shape))] = gsum[k].reshape(-1)
            (gco,), _ = O.clip_grads([flat_o.astype(np.float32)], CLIP, exact_norm=True)
            p2, m2u = O.rmsprop_update(p0, ms0, gco, LR)
            win["update_err_oracle_grad"] = [close_normscaled(pa - p0, p2 - p0, RTOL)[1],
                                             close_normscaled(ma, m2u, RTOL)[1]]
        res["windows"].append(win)
    if rank == 0:
        with open(os.path.join(outdir, "res.json"), "w") as f:
            json.dump(res, f, indent=1)
    else:
        with open(os.path.join(outdir, f"res{rank}.json"), "w") as f:
            json.dump(res, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
