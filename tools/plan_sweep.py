"""Tiling / replica-group planner sweep in one process: us/step of the bench window shape
(Philox, `warmup` untimed + `steps` timed iterations) per (workload, replicas, agents per
thread, replica groups).

    python tools/plan_sweep.py [--configs cfg3 cfg4] [--reps 4 8 16 32] [--apt 2 max] [--streams 1 2]

SPGG_APT is read by spgg_create, so it is set per engine here; `--reps N` takes the first N
replicas of the workload's grid (cycled with shifted seeds, as bench.py --replicas does)."""
import argparse
import dataclasses
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["cfg3", "cfg4"])
    ap.add_argument("--reps", nargs="+", type=int, default=[4, 8, 16, 32])
    ap.add_argument("--apt", nargs="+", default=["2", "max"])
    ap.add_argument("--streams", nargs="+", type=int, default=[1, 2])
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=100)
    a = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    for cfg in a.configs:
        desc, L, M2, state, grid = bench.workload(cfg, 0)
        for R in a.reps:
            reps = [dataclasses.replace(grid[i % len(grid)], seed=(grid[i % len(grid)].seed or 0) + 7919 * (i // len(grid)))
                    for i in range(R)]
            for apt in a.apt:
                for g in a.streams:
                    if g > R:
                        continue
                    os.environ["SPGG_APT"] = apt
                    eng = BatchEngine(L, a.steps + a.warmup, reps, use_second_order=M2, state_representation=state,
                                      rng="philox", streams=g)
                    eng.step(a.warmup)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    eng.step(a.steps)
                    torch.cuda.synchronize()
                    us = (time.perf_counter() - t0) / a.steps * 1e6
                    print(f"{cfg} R={R:3d} apt={apt:3s} groups={g} tile={eng.tile[0]}x{eng.tile[1]}: {us:7.2f} us/step "
                          f"{R * L * L / us * 1e6:.3g} agent-steps/s", flush=True)
                    eng.close()
    os.environ.pop("SPGG_APT", None)


if __name__ == "__main__":
    main()
