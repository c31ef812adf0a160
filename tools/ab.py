"""Interleaved in-process A/B timing of step-kernel builds (same ABI).

    python tools/ab.py --libs a.so b.so ... [--config cfg3] [--steps 200] [--warmup 20] [--rounds 3]

Each round builds a fresh engine per build (same workload, Philox), steps the
bench's warmup, then times the bench's window (iterations warmup+1 ..
warmup+steps, as bench.py does), in a rotating order; reports the median
us/step per build.  Variants must differ only in compile-time implementation
choices (SPGG_VARIANT / SPGG_ABLATE / SPGG_BLOCK ...)."""
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
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(args.config, 0)
    T = args.steps + args.warmup
    times = {p: [] for p in args.libs}
    for r in range(args.rounds):
        order = list(range(len(args.libs)))
        order = order[r % len(order):] + order[:r % len(order)]
        for i in order:
            eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng="philox",
                              lib_path=os.path.abspath(args.libs[i]))
            eng.step(args.warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step(args.steps)
            torch.cuda.synchronize()
            times[args.libs[i]].append((time.perf_counter() - t0) / args.steps * 1e6)
            eng.close()
    for p in args.libs:
        print(f"{os.path.basename(p):32s} median {statistics.median(times[p]):7.1f} us/step  "
              f"all {[round(x, 1) for x in times[p]]}")


if __name__ == "__main__":
    main()
