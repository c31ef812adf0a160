"""Per-iteration-window PMC counters of the step kernel from rocprofv3 passes over one run
(tools/window_probe.py --streams 1: dispatch k of spgg_step_kernel = iteration k).

    python tools/pmc_windows.py <dir> [--win 20] [--agents 4200000]

<dir> holds one subdirectory per --pmc pass (each with its counter_collection.csv and
kernel_trace.csv).  Prints, per window of iterations, the average of every counter per
dispatch and the kernel duration; FETCH_SIZE / WRITE_SIZE also as bytes per agent-step
(FETCH_SIZE doubled: gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md)."""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--win", type=int, default=20)
    ap.add_argument("--agents", type=float, default=4.2e6)
    ap.add_argument("--kernel", default="spgg_step_kernel")
    a = ap.parse_args()
    per = collections.defaultdict(dict)   # counter -> {dispatch order index: value}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if a.kernel in r["Kernel_Name"]]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        order = {d: i for i, d in enumerate(ids)}
        for r in rows:
            k = r["Counter_Name"]
            i = order[int(r["Dispatch_Id"])]
            per[k][i] = per[k].get(i, 0.0) + float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows = sorted((r for r in csv.DictReader(open(f)) if a.kernel in r["Kernel_Name"]),
                      key=lambda r: int(r["Start_Timestamp"]))
        for i, r in enumerate(rows):
            dur.setdefault(i, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    n = max([max(v) + 1 for v in per.values()] + [len(dur)])
    keys = sorted(per)
    head = "iters      dur_us " + " ".join(f"{k[:14]:>14s}" for k in keys)
    if "FETCH_SIZE" in per:
        head += "   rd_B/ag"
    if "WRITE_SIZE" in per:
        head += "   wr_B/ag"
    print(head)
    for lo in range(0, n, a.win):
        hi = min(n, lo + a.win)
        d = [x for i in range(lo, hi) for x in dur.get(i, [])]
        line = f"{lo + 1:4d}-{hi:<4d} {sum(d) / max(len(d), 1):8.2f} "
        vals = {}
        for k in keys:
            v = [per[k][i] for i in range(lo, hi) if i in per[k]]
            vals[k] = sum(v) / max(len(v), 1)
            line += f" {vals[k]:14.5g}"
        if "FETCH_SIZE" in vals:
            line += f"   {2 * vals['FETCH_SIZE'] * 1024 / a.agents:7.2f}"
        if "WRITE_SIZE" in vals:
            line += f"   {vals['WRITE_SIZE'] * 1024 / a.agents:7.2f}"
        print(line)


if __name__ == "__main__":
    main()
