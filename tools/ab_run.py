"""Interleaved in-process A/B of library builds (same ABI) over WHOLE runs: BatchEngine.run()
of a config (absorbing stops, host syncs, flush), in a rotating order; median us/iter per build.

    python tools/ab_run.py --libs a.so b.so [--config cfg3] [--rng mt19937] [--iters 2000] [--rounds 3]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rng", default="mt19937")
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--streams", type=int, default=None, help="replica groups (default: the planner's)")
    args = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(args.config, 0)
    times = {p: [] for p in args.libs}
    for r in range(args.rounds):
        order = list(range(len(args.libs)))
        order = order[r % len(order):] + order[:r % len(order)]
        for i in order:
            eng = BatchEngine(L, args.iters, reps, use_second_order=M2, state_representation=state, rng=args.rng,
                              lib_path=os.path.abspath(args.libs[i]), streams=args.streams)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(snapshots=False)
            torch.cuda.synchronize()
            times[args.libs[i]].append((time.perf_counter() - t0) / (eng.t - 1) * 1e6)
            print(f"  round {r} {args.libs[i]}: {times[args.libs[i]][-1]:.2f} us/iter", flush=True)
            eng.close()
    for p in args.libs:
        print(f"{args.config} {args.rng} {os.path.basename(p):24s} median {statistics.median(times[p]):7.2f} us/iter  "
              f"all {[round(x, 2) for x in times[p]]}", flush=True)


if __name__ == "__main__":
    main()
