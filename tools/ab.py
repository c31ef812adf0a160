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
    ap.add_argument("--clock", type=int, default=0,
                    help="us of a clock probe beside each timed window (tools/clock_probe.hip, "
                         "build_ablate/libclockprobe.so): the chip's effective clock, reported per build")
    args = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(args.config, 0)
    T = args.steps + args.warmup
    times = {p: [] for p in args.libs}
    mhz = {p: [] for p in args.libs}
    if args.clock:
        import ctypes
        clib = ctypes.CDLL(os.path.join(ROOT, "build_ablate", "libclockprobe.so"))
        clk = torch.zeros(2, dtype=torch.int64, device="cuda")
        cstream = torch.cuda.Stream()
    for r in range(args.rounds):
        order = list(range(len(args.libs)))
        order = order[r % len(order):] + order[:r % len(order)]
        for i in order:
            eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng="philox",
                              lib_path=os.path.abspath(args.libs[i]))
            eng.step(args.warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if args.clock:
                assert clib.clock_probe_launch(ctypes.c_void_p(clk.data_ptr()), 0, args.clock,
                                               ctypes.c_void_p(cstream.cuda_stream)) == 0
            eng.step(args.steps)
            torch.cuda.synchronize()
            times[args.libs[i]].append((time.perf_counter() - t0) / args.steps * 1e6)
            if args.clock:
                c = clk.cpu().tolist()
                mhz[args.libs[i]].append(c[0] / max(c[1], 1) * 100)
            eng.close()
    for p in args.libs:
        print(f"{os.path.basename(p):32s} median {statistics.median(times[p]):7.1f} us/step  "
              f"all {[round(x, 1) for x in times[p]]}"
              + (f"  MHz median {statistics.median(mhz[p]):.0f}" if mhz[p] else ""))


if __name__ == "__main__":
    main()
