"""Host-side cost of bench.py's timed window: wall time minus device time, by how the window's end
is awaited (torch.cuda.synchronize alone, or polling the end events first).

    python tools/sync_probe.py [--config cfg3] [--rounds 5]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    W, K = a.warmup, a.steps
    res = {"sync": [], "poll": []}
    for r in range(a.rounds):
        for mode in ("sync", "poll"):
            eng = BatchEngine(L, W + K, reps, use_second_order=M2, state_representation=state, rng="philox")
            eng.step(W)
            torch.cuda.synchronize()
            streams = eng.launch_streams()
            ev0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
            ev1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
            t0 = time.perf_counter()
            for e, s in zip(ev0, streams):
                e.record(s)
            eng.step(K, ordered=False)
            for e, s in zip(ev1, streams):
                e.record(s)
            t_enq = time.perf_counter() - t0
            if mode == "poll":
                while not all(e.query() for e in ev1):
                    pass
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            dev = max(x.elapsed_time(y) for x in ev0 for y in ev1) / 1e3
            res[mode].append((wall * 1e6 / K, dev * 1e6 / K, t_enq * 1e6))
            eng.close()
    print(desc)
    for m, v in res.items():
        print(f"{m}: wall {statistics.median(x[0] for x in v):.2f} device {statistics.median(x[1] for x in v):.2f} "
              f"us/step, host enqueue {statistics.median(x[2] for x in v):.0f} us  all {[tuple(round(y, 1) for y in x) for x in v]}")


if __name__ == "__main__":
    main()
