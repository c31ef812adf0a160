"""Where a whole run spends its time: BatchEngine.run() of a config timed per host turn
(the run's own 256-iteration turns; a device sync closes each), for one or more streams.

    python tools/fullrun_segments.py --config cfg3 [--rng philox mt19937] [--iters 10000]

Prints, per rng, the run's us/iter, then us/iter by 1000-iteration block of turns."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rng", nargs="+", default=["philox", "mt19937"])
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--block", type=int, default=1024)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    for rng in a.rng:
        eng = BatchEngine(L, a.iters, reps, use_second_order=M2, state_representation=state, rng=rng)
        marks = []
        try:
            torch.cuda.synchronize()

            def progress(t):
                torch.cuda.synchronize()
                marks.append((t, time.perf_counter()))

            t0 = time.perf_counter()
            marks.append((0, t0))
            eng.run(snapshots=False, progress=progress)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            layout = eng.mt_layout
        finally:
            eng.close()
        print(f"{a.config} {rng}: {wall / a.iters * 1e6:.2f} us/iter over {a.iters} iterations "
              f"(mt layout {layout})", flush=True)
        ts = np.array(marks)
        edges = list(range(0, a.iters + 1, a.block))
        line = []
        for lo, hi in zip(edges[:-1], edges[1:]):
            sel = (ts[:, 0] >= lo) & (ts[:, 0] <= hi)
            seg = ts[sel]
            if len(seg) >= 2:
                line.append(f"{int(seg[0, 0])}-{int(seg[-1, 0])}: "
                            f"{(seg[-1, 1] - seg[0, 1]) / max(seg[-1, 0] - seg[0, 0], 1) * 1e6:.1f}")
        print("  by block (us/iter): " + ", ".join(line), flush=True)
        d = np.diff(ts, axis=0)
        per = d[:, 1] / np.maximum(d[:, 0], 1) * 1e6
        print(f"  turns: first {per[0]:.1f}, median {np.median(per):.1f}, min {per.min():.1f}, "
              f"max {per.max():.1f} us/iter", flush=True)


if __name__ == "__main__":
    main()
