"""Time tools/stream_probe.hip: cost of each array's access width, no stencil."""
import ctypes
import os
import time

import torch

so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "build_ablate", "libsprobe.so")
lib = ctypes.CDLL(so)
d = torch.device("cuda")
n = 105 * 40000
Q = [torch.rand(n * 4, dtype=torch.float64, device=d) for _ in range(2)]
md = [torch.rand(n, dtype=torch.float64, device=d) for _ in range(2)]
atd = torch.rand(n, dtype=torch.float32, device=d)
S = [torch.zeros(n, dtype=torch.uint8, device=d) for _ in range(2)]
R = [torch.zeros(n, dtype=torch.int8, device=d) for _ in range(2)]
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(flags, K=100):
    def step(t):
        i, o = t & 1, (t + 1) & 1
        assert lib.sprobe_launch(*[ctypes.c_void_p(x.data_ptr()) for x in
                                   (Q[i], Q[o], md[i], md[o], atd, S[i], S[o], R[i], R[o])], n, flags, st) == 0
    for t in range(5):
        step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(K):
        step(t)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / K * 1e6
    per = (64 if flags & 1 else 0) + (16 if flags & 2 else 0) + (8 if flags & 4 else 0) + (4 if flags & 8 else 0)
    print(f"flags={flags:3d} {per:3d} B/agent: {us:6.1f} us  {n * per / us / 1e6:.2f} TB/s", flush=True)


for f in (1, 33, 2, 4, 8, 3, 7, 15, 18, 20, 24, 17, 31):
    run(f)
