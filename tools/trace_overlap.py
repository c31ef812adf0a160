"""Step-kernel launch durations split by what ran beside them, from a rocprofv3 --kernel-trace CSV
(e.g. of tools/fullrun_probe.py --rng mt19937): launches overlapping a generator launch
(spgg_mt_gen_kernel) vs launches with no generator beside them, and the per-iteration rate of
each regime (iterations completed per unit time).

    python tools/trace_overlap.py <dir> [--skip-first 512]"""
import argparse
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip-first", type=int, default=512)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    steps, gens, other = [], [], []
    for r in rows:
        iv = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        n = r["Kernel_Name"]
        (steps if "spgg_step" in n else gens if "mt_gen" in n else other).append(iv)
    steps.sort(); gens.sort()
    steps = steps[a.skip_first:]
    t0 = steps[0][0]
    t1 = max(e for _, e in steps)
    gens = [g for g in gens if g[1] > t0 and g[0] < t1]
    def gen_frac(s, e):
        ov = sum(max(0, min(e, ge) - max(s, gs)) for gs, ge in gens)
        return ov / (e - s)
    with_g = [(e - s) / 1e3 for s, e in steps if gen_frac(s, e) > 0.5]
    without = [(e - s) / 1e3 for s, e in steps if gen_frac(s, e) == 0.0]
    gbusy = sum(min(e, t1) - max(s, t0) for s, e in gens) / (t1 - t0)
    print(f"window {(t1 - t0) / 1e3:.1f} us, {len(steps)} step launches, generator busy {gbusy * 100:.0f} %")
    for name, v in (("beside generator", with_g), ("alone", without)):
        if v:
            print(f"  step launches {name:17s}: n={len(v):5d} mean {statistics.mean(v):6.2f} median {statistics.median(v):6.2f} us")
    if gens:
        d = [(e - s) / 1e3 for s, e in gens]
        print(f"  generator launches: n={len(d)} mean {statistics.mean(d):.1f} us")
    # per-iteration rate while the generator runs vs not: step launches ENDING in each regime
    ends_g = sum(1 for s, e in steps if any(gs <= e <= ge for gs, ge in gens))
    tg = gbusy * (t1 - t0) / 1e3
    print(f"  launches ending beside the generator: {ends_g} in {tg:.0f} us -> {tg / max(ends_g, 1):.2f} us per launch; "
          f"otherwise {len(steps) - ends_g} in {(t1 - t0) / 1e3 - tg:.0f} us -> "
          f"{((t1 - t0) / 1e3 - tg) / max(len(steps) - ends_g, 1):.2f}")


if __name__ == "__main__":
    main()
