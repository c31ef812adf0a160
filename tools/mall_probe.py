"""Bandwidth of in-place vs out-of-place f64 streams by footprint (does the MI355X
infinity cache (MALL) keep a ping-ponged or in-place working set resident?)."""
import time

import torch

d = torch.device("cuda")


def bench(fn, K=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6


for mb in (32, 64, 100, 134, 180, 256, 400, 538):
    n = mb * 1024 * 1024 // 8
    a = torch.rand(n, dtype=torch.float64, device=d)
    b = torch.empty_like(a)
    us_in = bench(lambda: a.mul_(1.0000001))
    us_cp = bench(lambda: b.copy_(a))
    byts = 2 * n * 8
    print(f"{mb:4d} MB  in-place {us_in:7.1f} us {byts / us_in / 1e6:5.2f} TB/s   "
          f"copy {us_cp:7.1f} us {byts / us_cp / 1e6:5.2f} TB/s", flush=True)
    del a, b
