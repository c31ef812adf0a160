"""Per-iteration launch spans of the step kernel from a rocprofv3 --kernel-trace CSV of one run
(tools/window_probe.py): launch k of each stream = iteration k.

    python tools/trace_windows.py <dir> [--win 20] [--groups 2]

Per window of iterations: mean launch duration per group, and the iteration period (start of
iteration t+1's first launch - start of iteration t's first launch)."""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--win", type=int, default=20)
    ap.add_argument("--kernel", default="spgg_step_kernel")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if a.kernel in r["Kernel_Name"]]
    by_q = collections.defaultdict(list)
    for r in rows:
        by_q[r.get("Stream_Id") or r.get("Queue_Id")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    qs = sorted(by_q, key=lambda q: min(by_q[q])[0])
    for q in qs:
        by_q[q].sort()
    n = min(len(by_q[q]) for q in qs)
    print(f"streams {len(qs)}, iterations {n}")
    print("iters       " + " ".join(f"dur_q{i:<5d}" for i in range(len(qs))) + "  period_us  overlap_us")
    for lo in range(0, n - 1, a.win):
        hi = min(n - 1, lo + a.win)
        durs = [sum((by_q[q][i][1] - by_q[q][i][0]) for i in range(lo, hi)) / (hi - lo) / 1e3 for q in qs]
        period = (min(by_q[q][hi][0] for q in qs) - min(by_q[q][lo][0] for q in qs)) / (hi - lo) / 1e3
        ov = 0.0
        if len(qs) == 2:
            for i in range(lo, hi):
                (s0, e0), (s1, e1) = by_q[qs[0]][i], by_q[qs[1]][i]
                ov += max(0, min(e0, e1) - max(s0, s1))
            ov /= (hi - lo) * 1e3
        print(f"{lo + 1:4d}-{hi:<5d} " + " ".join(f"{d:10.2f}" for d in durs) + f"  {period:9.2f}  {ov:9.2f}")


if __name__ == "__main__":
    main()
