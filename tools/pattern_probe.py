"""Time tools/pattern_probe.hip: which part of the step kernel's traffic pattern costs what.
    python tools/pattern_probe.py   (build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC
                                     tools/pattern_probe.hip -o build_ablate/libpprobe.so)"""
import ctypes
import os
import time

import torch

so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "build_ablate", "libpprobe.so")
lib = ctypes.CDLL(so)
d = torch.device("cuda")


def run(R, flags, G=1, L=200, TW=40, TH=25, K=100):
    n = L * L if not flags & 64 else ((L + TW - 1) // TW) * ((L + TH - 1) // TH) * 1024
    S = [torch.zeros((R, n), dtype=torch.uint8, device=d) for _ in range(2)]
    Rr = [torch.zeros((R, n), dtype=torch.int8, device=d) for _ in range(2)]
    Q = [torch.rand((R, n, 6 if flags & 16 else 4), dtype=torch.float64, device=d) for _ in range(2)]
    md = [torch.rand((R, n), dtype=torch.float64, device=d) for _ in range(2)]
    atd = torch.rand((R, n), dtype=torch.float32, device=d)
    bounds = [R * g // G for g in range(G + 1)]
    streams = [torch.cuda.current_stream()] if G == 1 else [torch.cuda.Stream() for _ in range(G)]
    main = torch.cuda.current_stream()

    def step(t):
        i, o = (t - 1) & 1, t & 1
        for g in range(G):
            r0, r1 = bounds[g], bounds[g + 1]
            s = streams[g]
            rc = lib.pprobe_launch(*[ctypes.c_void_p(x[r0].data_ptr()) for x in
                                     (S[i], S[o], Rr[i], Rr[o], Q[i], Q[o], md[i], md[o], atd)],
                                   L, TW, TH, r1 - r0, flags, ctypes.c_void_p(s.cuda_stream))
            assert rc == 0

    def run_steps(a, b):
        if G > 1:
            for s in streams:
                s.wait_stream(main)
        for t in range(a, b):
            step(t)
        if G > 1:
            for s in streams:
                main.wait_stream(s)

    run_steps(1, 6)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(6, 6 + K)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / K * 1e6
    per = 64 + ((32 if flags & 16 else 24) if flags & 2 else 0) + (4 if flags & 4 else 0)
    print(f"R={R:4d} G={G} flags={flags:2d} ({per:3d} B/agent): {us:6.1f} us  "
          f"{R * L * L * per / us / 1e6:.2f} TB/s", flush=True)


for G in (1, 6):
    for flags in (1, 3, 5, 7, 65, 67, 69, 71):
        run(105, flags, G)
