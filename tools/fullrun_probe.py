"""Whole-run timing (bench.full_run) of one config in a fresh process, optionally after a
bench-shaped engine (--after-bench: the state bench.py leaves behind), to tell stream /
hardware-queue effects from the kernels.

    python tools/fullrun_probe.py --config cfg3 --rng mt19937 [--iters 3000] [--after-bench]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rng", default="mt19937")
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--after-bench", action="store_true")
    ap.add_argument("--repeat", type=int, default=1)
    ap.add_argument("--turn", type=int, default=256, help="iterations between host syncs (BatchEngine.run chunk)")
    a = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    if a.after_bench:
        eng = BatchEngine(L, 60, reps, use_second_order=M2, state_representation=state, rng=a.rng)
        eng.step(60)
        torch.cuda.synchronize()
        eng.close()
    for i in range(a.repeat):
        r = bench.full_run(L, M2, state, reps, a.rng, None, a.iters, 0, a.turn)
        print(f"{a.config} {a.rng} turn={a.turn} after_bench={a.after_bench} run {i}: {r['seconds'] / a.iters * 1e6:.2f} us/iter "
              f"({r['value']:.3g} agent-steps/s)", flush=True)


if __name__ == "__main__":
    main()
