"""Per-iteration completion times inside a short timed window (where does a 20-iteration window
lose its ~150 us over the long-window rate?).

    python tools/window_timeline.py [--config cfg3] [--warmup 5] [--steps 20] [--rounds 3]

A fresh engine steps the warm-up, synchronises, then enqueues the window one iteration at a time
(spgg_step_groups, every group) with a HIP event recorded on every group stream after each
iteration; completion of iteration k = the latest of its groups' events, relative to the event
opening the window (recorded on the current stream, which the groups wait for, as bench.py does).
Also times the same window without the per-iteration events (their own cost)."""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from spgg_amd import _lib as C
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    W, K = a.warmup, a.steps
    print(desc, f"window {W + 1}-{W + K}", flush=True)
    for r in range(a.rounds):
        for mode in ("startwait", "endwait", "bothwait_side"):
            # one of the two cross-stream dependencies only, or both on a non-default current stream
            eng = BatchEngine(L, W + K, reps, use_second_order=M2, state_representation=state, rng="philox")
            eng.step(W)
            torch.cuda.synchronize()
            live = eng.groups
            ctxs = (ctypes.c_void_p * len(live))(*[g["ctx"] for g in live])
            strs = (ctypes.c_void_p * len(live))(*[g["stream"].cuda_stream for g in live])
            side = torch.cuda.Stream()
            cur = side if mode == "bothwait_side" else torch.cuda.current_stream()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode != "endwait":
                for g in live:
                    g["stream"].wait_stream(cur)
            C.check(eng.lib.spgg_step_groups(ctxs, strs, len(live), W + 1, K), live[0]["ctx"], "step")
            if mode != "startwait":
                for g in live:
                    cur.wait_stream(g["stream"])
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e6
            print(f"round {r} {mode}: wall {wall / K:.2f} us/step", flush=True)
            eng.close()
        for mode in ("nowait", "nowait_wall"):
            # the groups' streams do NOT wait for the current stream (idle after the sync anyway):
            # a start and an end event on every group stream, window = last end - first start
            eng = BatchEngine(L, W + K, reps, use_second_order=M2, state_representation=state, rng="philox")
            eng.step(W)
            torch.cuda.synchronize()
            live = eng.groups
            ctxs = (ctypes.c_void_p * len(live))(*[g["ctx"] for g in live])
            strs = (ctypes.c_void_p * len(live))(*[g["stream"].cuda_stream for g in live])
            st = [torch.cuda.Event(enable_timing=True) for _ in live]
            en = [torch.cuda.Event(enable_timing=True) for _ in live]
            t0 = time.perf_counter()
            if mode == "nowait":
                for e, g in zip(st, live):
                    e.record(g["stream"])
            C.check(eng.lib.spgg_step_groups(ctxs, strs, len(live), W + 1, K), live[0]["ctx"], "step")
            if mode == "nowait":
                for e, g in zip(en, live):
                    e.record(g["stream"])
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e6
            if mode == "nowait":
                dev = max(st[i].elapsed_time(en[j]) for i in range(len(live)) for j in range(len(live))) * 1e3
                print(f"round {r} no cross-stream wait: device {dev / K:.2f} us/step, wall {wall / K:.2f} us/step",
                      flush=True)
            else:
                print(f"round {r} no cross-stream wait, no events: wall {wall / K:.2f} us/step", flush=True)
            eng.close()
        for per_iter in (True, False):
            eng = BatchEngine(L, W + K, reps, use_second_order=M2, state_representation=state, rng="philox")
            eng.step(W)
            torch.cuda.synchronize()
            live = eng.groups
            ctxs = (ctypes.c_void_p * len(live))(*[g["ctx"] for g in live])
            strs = (ctypes.c_void_p * len(live))(*[g["stream"].cuda_stream for g in live])
            cur = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            evs = []
            t0 = time.perf_counter()
            e0.record(cur)
            for g in live:
                g["stream"].wait_stream(cur)
            if per_iter:
                for k in range(K):
                    C.check(eng.lib.spgg_step_groups(ctxs, strs, len(live), W + 1 + k, 1), live[0]["ctx"], "step")
                    row = []
                    for g in live:
                        ev = torch.cuda.Event(enable_timing=True)
                        ev.record(g["stream"])
                        row.append(ev)
                    evs.append(row)
            else:
                C.check(eng.lib.spgg_step_groups(ctxs, strs, len(live), W + 1, K), live[0]["ctx"], "step")
            for g in live:
                cur.wait_stream(g["stream"])
            e1.record(cur)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e6
            tot = e0.elapsed_time(e1) * 1e3
            if per_iter:
                done = np.array([[e0.elapsed_time(ev) * 1e3 for ev in row] for row in evs])
                fin = done.max(axis=1)
                d = np.diff(np.concatenate([[0.0], fin]))
                print(f"round {r} per-iteration events: total {tot:.1f} us = {tot / K:.2f} us/step; "
                      f"iteration deltas (us): {' '.join(f'{x:.0f}' for x in d)}", flush=True)
                print(f"   groups' completion skew (us): {' '.join(f'{x:.0f}' for x in done.max(1) - done.min(1))}",
                      flush=True)
            else:
                print(f"round {r} no events: total {tot:.1f} us = {tot / K:.2f} us/step, wall {wall / K:.2f}", flush=True)
            eng.close()


if __name__ == "__main__":
    main()
