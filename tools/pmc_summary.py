"""Summarise rocprofv3 --pmc CSVs for one kernel: python tools/pmc_summary.py <dir> [kernel-substr]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "spgg_step"
agg = collections.defaultdict(list)
dur = []
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {k: sum(v) / len(v) for k, v in agg.items()}
for k in sorted(out):
    print(f"{k:24s} {out[k]:.4g}")
if dur:
    print(f"{'avg_duration_us':24s} {sum(dur) / len(dur) / 1e3:.2f}  (n={len(dur)})")
if "SQ_WAVE_CYCLES" in out:
    wc = out["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in out:
            print(f"  {k}/WAVE_CYCLES = {out[k] / wc:.2f}")
if "SQ_WAVES" in out and "SQ_INSTS_VALU" in out:
    print(f"  VALU insts per wave = {out['SQ_INSTS_VALU'] / out['SQ_WAVES']:.0f}")
if "FETCH_SIZE" in out:
    print(f"  FETCH_SIZE x2 (gfx950 correction) = {2 * out['FETCH_SIZE'] * 1024 / 1e6:.1f} MB per launch")
if "WRITE_SIZE" in out:
    print(f"  WRITE_SIZE = {out['WRITE_SIZE'] * 1024 / 1e6:.1f} MB per launch")
