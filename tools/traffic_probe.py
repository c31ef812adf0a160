"""Time the memory-only probe (tools/traffic_probe.hip): tiling / round / write effects."""
import ctypes
import os
import time

import torch

so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "build_ablate", "libprobe.so")
lib = ctypes.CDLL(so)
d = torch.device("cuda")
st = torch.cuda.current_stream().cuda_stream


def run(R, TW, TH, mode, L=200, K=100):
    n = L * L
    S = [torch.zeros((R, n), dtype=torch.uint8, device=d) for _ in range(2)]
    Rr = [torch.zeros((R, n), dtype=torch.int8, device=d) for _ in range(2)]
    Q = [torch.rand((R, n, 4), dtype=torch.float64, device=d) for _ in range(2)]
    md = [torch.rand((R, n), dtype=torch.float64, device=d) for _ in range(2)]
    atd = torch.rand((R, n), dtype=torch.float32, device=d)

    def step(t):
        i, o = (t - 1) & 1, t & 1
        rc = lib.probe_launch(*[ctypes.c_void_p(x.data_ptr()) for x in
                                (S[i], S[o], Rr[i], Rr[o], Q[i], Q[o], md[i], md[o], atd)],
                              L, TW, TH, R, mode, ctypes.c_void_p(st))
        assert rc == 0

    for t in range(1, 6):
        step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(6, 6 + K):
        step(t)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / K * 1e6
    byts = R * n * (32 + 8 + 4 + 1 + 1) * (1 if mode & 1 else 2)
    tiles = ((L + TW - 1) // TW) * ((L + TH - 1) // TH) * R
    print(f"R={R:4d} tile={TW}x{TH} mode={mode} tiles={tiles:5d} rounds={tiles / 1024:5.2f}: "
          f"{us:6.1f} us  {byts / us / 1e6:.2f} TB/s", flush=True)
    del S, Rr, Q, md, atd


import sys
if "--copy" in sys.argv:  # plain device copy of the same Q bytes (read+write bandwidth reference)
    for R in (105, 420):
        a = torch.rand((R, 40000, 4), dtype=torch.float64, device=d)
        b = torch.empty_like(a)
        for _ in range(5):
            b.copy_(a)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(100):
            b.copy_(a)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / 100 * 1e6
        print(f"copy R={R}: {us:.1f} us  {2 * a.numel() * 8 / us / 1e6:.2f} TB/s", flush=True)
for R in (26, 52, 105, 210, 420):
    run(R, 40, 25, 0)
    run(R, 40, 25, 2)
