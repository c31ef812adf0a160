"""Does launch overhead matter for the latency-bound shapes?  Eager step launches vs the same
launches captured in a HIP graph and replayed.

    python tools/graph_probe.py --config cfg2 [--steps 200] [--warmup 400] [--rounds 3]

Philox (the kernels go to one stream; G = 1 for the single-replica configs).  Per round: a fresh
engine steps `warmup` iterations eagerly, then times `steps` more eagerly; a second fresh engine
steps `warmup` eagerly, captures the next `steps` launches into a graph (torch.cuda.graph on
torch's capture stream, which spgg_step enqueues on), and times one replay.  The replay re-runs
those launches' iteration numbers over the state the capture left (the timing, not the science,
is what is compared)."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    T = a.warmup + 2 * a.steps
    res = {"eager": [], "graph": []}
    for _ in range(a.rounds):
        eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng="philox", streams=1)
        eng.step(a.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step(a.steps)
        torch.cuda.synchronize()
        res["eager"].append((time.perf_counter() - t0) / a.steps * 1e6)
        eng.close()
        eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng="philox", streams=1)
        eng.step(a.warmup)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            eng.step(a.steps)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        res["graph"].append((time.perf_counter() - t0) / a.steps * 1e6)
        del g
        eng.close()
    for k, v in res.items():
        print(f"{a.config} {k:5s}: median {statistics.median(v):6.2f} us/iter  all {[round(x, 2) for x in v]}",
              flush=True)


if __name__ == "__main__":
    main()
