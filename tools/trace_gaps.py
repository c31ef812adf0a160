"""Idle gaps of the step-kernel streams and the generator's launches, from a rocprofv3
--kernel-trace CSV (e.g. of tools/fullrun_probe.py --rng mt19937): are the steps waiting for draws?

    python tools/trace_gaps.py <dir> [--skip-first 512]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip-first", type=int, default=512, help="step launches (all streams) to skip")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    ks = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        kind = "step" if "spgg_step" in name else "gen" if "mt_gen" in name else "jump" if "mt_jump" in name else None
        if kind:
            ks[(kind, r["Queue_Id"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k in ks:
        ks[k].sort()
    steps = sorted((k for k in ks if k[0] == "step"), key=lambda k: ks[k][0][0])
    t_from = sorted(s for k in steps for s, _ in ks[k])[a.skip_first] if steps else 0
    t_to = max(e for k in ks for _, e in ks[k])
    span = (t_to - t_from) / 1e3
    print(f"window {span:.1f} us from step launch {a.skip_first}")
    for k in sorted(ks):
        iv = [(s, e) for s, e in ks[k] if s >= t_from]
        if not iv:
            continue
        busy = sum(e - s for s, e in iv) / 1e3
        gaps = [(iv[i + 1][0] - iv[i][1]) / 1e3 for i in range(len(iv) - 1)]
        big = sorted(gaps)[-5:] if gaps else []
        print(f"{k[0]:5s} queue {k[1]}: {len(iv)} launches, busy {busy:.1f} us ({busy / span * 100:.0f} %), "
              f"mean {busy / len(iv):.2f} us, gaps sum {sum(gaps):.1f} us, largest {[round(g, 1) for g in big]}")


if __name__ == "__main__":
    main()
