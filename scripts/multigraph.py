"""Env-group chains as one multi-stream graph vs one single-stream graph per
chain (diagnostic): the window = chain graphs replayed on their own streams,
then the learner graph after both.  Reports ms/window for both forms and the
host time of the launches.  python scripts/multigraph.py [c4|c3] [groups]"""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT]
import bench  # noqa: E402


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "c4"
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    pkg = bench._import_pkg()
    dev = torch.device("cuda", 0)
    arch, N, A = bench.WORKLOADS[w]
    T, P = 5, 64
    Model = pkg.A3CLSTM if arch == "lstm" else pkg.A3CFF
    model = Model(A, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev, frames="pairs")
    opt = pkg.RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(pkg.GradientClipping(40))
    ag = pkg.A3C(model, opt, T, 0.99, beta=1e-2)
    pairs, rewards, dones = bench.synth_pools(N, P, 0, dev)
    net = model.net
    groups = net.env_groups(G)
    streams = [torch.cuda.Stream(device=dev) for _ in groups]
    s0 = streams[0]
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        ag.run_window(pairs, rewards, dones, P, first=True, stream=s0, env_groups=G)
        ag.run_window(pairs, rewards, dones, P, stream=s0, env_groups=G)
        s0.synchronize()
        # (a) one multi-stream graph (what the bench captures)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s0):
            ag.run_window(pairs, rewards, dones, P, stream=s0, env_groups=G)
        s0.synchronize()
    # (b) one graph per chain + the learner graph
    cg = []
    for envs, s in zip(groups, streams):
        s.wait_stream(s0)
        with torch.cuda.stream(s):
            gg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gg, stream=s):
                ag._forward_chain(pairs, rewards, dones, P, False, s, envs)
            cg.append(gg)
        s.synchronize()
    with torch.cuda.stream(s0):
        lg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(lg, stream=s0):
            ag._learn(s0)
            ag.finish_window(stream=s0)
    torch.cuda.synchronize()

    def win_a():
        g.replay()

    def win_b():
        for s in streams[1:]:
            s.wait_stream(s0)
        for gg, s in zip(cg, streams):
            with torch.cuda.stream(s):
                gg.replay()
        for s in streams[1:]:
            s0.wait_stream(s)
        lg.replay()

    K = 100
    res = {}
    for name, fn in (("multi-stream graph", win_a), ("graph per chain", win_b)) * 2:
        with torch.cuda.stream(s0):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                fn()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        res[name] = (1e3 * (t1 - t0) / K, 1e3 * (t2 - t0) / K)
        print(f"{w} G={G} {name}: host {res[name][0]:.4f} ms/window, wall {res[name][1]:.4f} ms/window", flush=True)


if __name__ == "__main__":
    main()
