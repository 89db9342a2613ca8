"""Host-side cost of one window graph replay (diagnostic): builds the bench's
agent for a workload, captures one window, then times K replays (a) the host
time of the replay() calls alone, no sync, (b) wall time with a final sync,
(c) replays each followed by a sync.  If (a) ~ (b), the host submission of
the graph's nodes paces the GPU.
  python scripts/replay_host.py [c4|c3|c2] [env_groups]"""
import os
import sys
import time

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT]
import bench  # noqa: E402


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "c4"
    groups = int(sys.argv[2]) if len(sys.argv) > 2 else None
    pkg = bench._import_pkg()
    dev = torch.device("cuda", 0)
    arch, N, A = bench.WORKLOADS[w]
    T, P = 5, 64
    Model = pkg.A3CLSTM if arch == "lstm" else pkg.A3CFF
    model = Model(A, n_envs=N, t_max=T, seed=1, init_seed=0, device=dev, frames="pairs")
    opt = pkg.RMSpropAsync(lr=7e-4, eps=1e-1, alpha=0.99).setup(model)
    opt.add_hook(pkg.GradientClipping(40))
    agent = pkg.A3C(model, opt, T, 0.99, beta=1e-2)
    pairs, rewards, dones = bench.synth_pools(N, P, 0, dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        agent.run_window(pairs, rewards, dones, P, first=True, stream=s, env_groups=groups)
        agent.run_window(pairs, rewards, dones, P, stream=s, env_groups=groups)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            agent.run_window(pairs, rewards, dones, P, stream=s, env_groups=groups)
        for _ in range(5):
            g.replay()
    s.synchronize()
    K = 50
    with torch.cuda.stream(s):
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        t1 = time.perf_counter()
        s.synchronize()
        t2 = time.perf_counter()
        lat = []
        for _ in range(20):
            a = time.perf_counter()
            g.replay()
            b = time.perf_counter()
            s.synchronize()
            c = time.perf_counter()
            lat.append((b - a, c - a))
    lat.sort(key=lambda x: x[1])
    med = lat[len(lat) // 2]
    print(f"{w} groups={groups}: host replay() {1e3 * (t1 - t0) / K:.4f} ms/window, "
          f"wall {1e3 * (t2 - t0) / K:.4f} ms/window; single replay: call {1e3 * med[0]:.4f} ms, "
          f"call+sync {1e3 * med[1]:.4f} ms")


if __name__ == "__main__":
    main()
