"""Do two torch streams captured into one torch.cuda.CUDAGraph run
concurrently?  Chains of torch.cuda._sleep spin kernels, serial vs forked,
graph vs eager (companion of graph_branches.hip, which captures with raw HIP).
"""
import time

import torch

K, CYC = 50, 20000


def chain(main, side, forked):
    if forked:
        side.wait_stream(main)
    for _ in range(K):
        with torch.cuda.stream(main):
            torch.cuda._sleep(CYC)
        with torch.cuda.stream(side if forked else main):
            torch.cuda._sleep(CYC)
    if forked:
        main.wait_stream(side)


def timeit(fn, reps=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / (2 * K) * 1e6


main, side = torch.cuda.Stream(), torch.cuda.Stream()
for forked in (False, True):
    print({"mode": "eager", "forked": forked, "us_per_kernel": round(timeit(lambda: chain(main, side, forked)), 3)})
    g = torch.cuda.CUDAGraph()
    main.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=main):
        chain(main, side, forked)
    g.replay()
    print({"mode": "graph", "forked": forked, "us_per_kernel": round(timeit(g.replay), 3)})
