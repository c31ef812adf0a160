"""Time the MT19937 draw generator alone (spgg_draw, one iteration per launch, and the
pipelined chunk launches of spgg_step's generator), per library build.

    python tools/mt_gen_probe.py [--L 200] [--reps 1 105] [--iters 40] [--libs a.so b.so]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=200)
    ap.add_argument("--reps", type=int, nargs="+", default=[1, 105])
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--libs", nargs="+", default=[None])
    args = ap.parse_args()
    import numpy as np
    import torch
    import spgg_amd  # noqa: F401
    from spgg_amd import _lib as C
    from spgg_amd.engine import BatchEngine, ReplicaParams
    for lib in args.libs:
        for R in args.reps:
            reps = [ReplicaParams(r=3.0, seed=s, epsilon=0.5, epsilon_decay=0.99) for s in range(R)]
            eng = BatchEngine(args.L, args.iters + 2, reps, use_second_order=False, rng="mt19937",
                              lib_path=lib, streams=1)
            st = torch.cuda.current_stream()
            for t in (1, 2):
                C.check(eng.lib.spgg_draw(eng.ctx, t, st.cuda_stream), eng.ctx, "spgg_draw")
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for t in range(3, args.iters + 3):
                eng.lib.spgg_draw(eng.ctx, t, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            words = 3 * args.L * args.L
            print(f"lib={os.path.basename(lib or 'in-tree')} L={args.L} reps={R}: {us:.1f} us/iteration "
                  f"({words / us / 1e3:.2f} Gwords/s per replica)", flush=True)
            eng.close()


if __name__ == "__main__":
    main()
