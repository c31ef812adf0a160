"""Step time by iteration window: where a run's early iterations lose time.

    python tools/window_probe.py [--config cfg3] [--upto 600] [--win 20] [--preheat 0]

A fresh engine steps `--win` iterations at a time from iteration 1; each window is
bracketed by HIP events on the current stream (the engine orders every replica group's
launches between them).  --preheat N first runs N iterations of another engine (the
GPU's clocks and caches busy before the measured engine starts).  Prints us/iter per
window with the window's mean switch rate and eps (what changes with the dynamics)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rng", default="philox")
    ap.add_argument("--upto", type=int, default=600)
    ap.add_argument("--win", type=int, default=20)
    ap.add_argument("--first", type=int, default=0, help="untimed iterations before the first window")
    ap.add_argument("--preheat", type=int, default=0)
    ap.add_argument("--streams", type=int, default=None)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--hot-ms", type=float, default=0.0,
                    help="after making the measured engine, keep the GPU streaming memory for this many "
                         "ms (torch copies of a 1 GiB buffer) right before the first window")
    ap.add_argument("--clock", type=int, default=0,
                    help="us of a clock probe (build_ablate/libclockprobe.so, tools/clock_probe.hip) run on "
                         "its own stream beside each window: the chip's effective clock in that window")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from spgg_amd import _lib as C
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    if a.preheat:
        pre = [type(p)(**{**p.__dict__, "seed": (p.seed or 0) + 500}) for p in reps]
        e0 = BatchEngine(L, a.preheat, pre, use_second_order=M2, state_representation=state, rng=a.rng,
                         streams=a.streams, lib_path=a.lib)
        t0 = time.perf_counter()
        e0.step(a.preheat)
        torch.cuda.synchronize()
        print(f"preheat: {a.preheat} iterations, {(time.perf_counter() - t0) / a.preheat * 1e6:.1f} us/iter",
              flush=True)
        e0.close()
    eng = BatchEngine(L, a.upto + a.first, reps, use_second_order=M2, state_representation=state, rng=a.rng,
                      streams=a.streams, lib_path=a.lib)
    if a.hot_ms > 0:
        buf = torch.empty(2 ** 27, dtype=torch.float64, device="cuda")
        dst = torch.empty_like(buf)
        torch.cuda.synchronize()
        t_end = time.perf_counter() + a.hot_ms / 1e3
        while time.perf_counter() < t_end:
            for _ in range(4):
                dst.copy_(buf)
            torch.cuda.synchronize()
        del buf, dst
    if a.first:
        eng.step(a.first)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    evs = []
    clk = None
    if a.clock:
        import ctypes
        clib = ctypes.CDLL(os.path.join(ROOT, "build_ablate", "libclockprobe.so"))
        nwin = -(-a.upto // a.win)
        clk = torch.zeros(2 * nwin, dtype=torch.int64, device="cuda")
        cstream = torch.cuda.Stream()
    t = a.first
    while t < a.upto + a.first:
        k = min(a.win, a.upto + a.first - t)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        if clk is not None:
            cstream.wait_event(e0)
            assert clib.clock_probe_launch(ctypes.c_void_p(clk.data_ptr()), len(evs), a.clock,
                                           ctypes.c_void_p(cstream.cuda_stream)) == 0
        eng.step(k)
        e1.record(cur)
        torch.cuda.synchronize()   # one window in flight at a time (as the bench's timed region)
        if clk is not None:
            torch.cuda.synchronize()
        evs.append((t + 1, k, e0.elapsed_time(e1)))
        t += k
    st = eng.stats_folded().cpu().numpy()
    n = L * L
    print(f"{desc} ({a.rng}, groups {eng.G}, streams {eng.resident}, apt/tile {eng.tile})", flush=True)
    clocks = clk.view(-1, 2).cpu().numpy() if clk is not None else None
    print("window      us/iter   eps     switches/agent  coop" + ("    MHz" if clk is not None else ""), flush=True)
    for w, (t0, k, ms) in enumerate(evs):
        sl = slice(t0, t0 + k)
        sw = (st[:, sl, C.ST_SW_CD].sum() * 2 + 0.0) / (len(reps) * k * n)
        coop = st[:, sl, C.ST_NCOOP].mean() / n
        mhz = f"  {clocks[w, 0] / max(clocks[w, 1], 1) * 100:7.0f}" if clocks is not None else ""
        print(f"{t0:4d}-{t0 + k - 1:<5d} {ms * 1e3 / k:8.2f}  {eng.eps_host[0, t0]:.4f}  {sw:10.4f}  {coop:8.4f}{mhz}",
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
