"""RMSProp kernel (arl_rmsprop, clip off: 20 B / param) and the HBM stream copy
(arl_stream_copy, one-shot non-temporal form) over the same byte counts, from
the FF net's 677k parameters up to 64M: time per launch between HIP events
over back-to-back launches, and the achieved GB/s.  Shows where the update is
latency-bound (small) and where it streams at the HBM rate (large).
    python scripts/rms_sweep.py [out.json]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "async-rl_amd")]
from asyncrl_amd._lib import check, lib, ptr  # noqa: E402


def timed(fn, reps=200, warm=20):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps   # us per launch


def main(out=None):
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    rows = []
    for n in (677_429, 2 ** 21, 2 ** 23, 2 ** 25, 2 ** 26):
        p = torch.randn(n, device=dev) * 0.01
        ms = torch.rand(n, device=dev)
        g = torch.randn(n, device=dev)
        us = timed(lambda: check(lib.arl_rmsprop(ptr(p), ptr(ms), ptr(g), n, 1e-9, 0.99, 0.1, 0.0, None, s)))
        nb = 20 * n
        # the same bytes as a copy: read 12 n, write 8 n -> a copy of 10 n bytes moves 20 n
        cb = (10 * n) // 16 * 16
        src = torch.empty(cb // 4, device=dev)
        dst = torch.empty_like(src)
        cus = timed(lambda: check(lib.arl_stream_copy(ptr(src), ptr(dst), cb, 0, 3, s)))
        rows.append({"params": n, "bytes": nb, "rmsprop_us": round(us, 3), "rmsprop_GBs": round(nb / us / 1e3, 1),
                     "copy_same_bytes_us": round(cus, 3), "copy_GBs": round(2 * cb / cus / 1e3, 1)})
        print(json.dumps(rows[-1]), flush=True)
        del p, ms, g, src, dst
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
