"""HBM-traffic figure for bench.py from separate rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes of the same command (MI355X_MICROARCH.md, HBM section):

    python tools/traffic_json.py <round-dir> <agents-per-launch> <config> <streams> [window] [skip]
        > traffic_<config>[_w<window>].json

window: the bench window the passes ran ("6-25"), recorded in the file; skip: step-kernel
dispatches (in dispatch order) before the window's, left out of the averages (the warm-up's).

FETCH_SIZE is doubled (gfx950 reports half of wide streaming reads); both
counters are in KiB per dispatch; Infinity-Cache hits are counted by these
memory-side counters."""
import csv
import glob
import json
import os
import sys

d, agents, cfg, streams = sys.argv[1], float(sys.argv[2]), sys.argv[3], int(sys.argv[4])
window = sys.argv[5] if len(sys.argv) > 5 else None
skip = int(sys.argv[6]) if len(sys.argv) > 6 else 0
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    per = {}
    for r in csv.DictReader(open(f)):
        if "spgg_step" in r["Kernel_Name"] and r["Counter_Name"] in vals:
            k = (r["Counter_Name"], int(r["Dispatch_Id"]))
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    for name in vals:
        ids = sorted(i for (c, i) in per if c == name)
        vals[name] += [per[(name, i)] for i in ids[skip:]]
fetch = 2 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"]) * 1024
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"]) * 1024
print(json.dumps({
    "config": cfg, "window": window, "skipped_dispatches": skip, "streams": streams, "agents_per_launch": agents,
    "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
    "bytes_per_agent_step": (fetch + write) / agents,
    "dispatches": {k: len(v) for k, v in vals.items()},
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE doubled "
              "(gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md HBM); KiB x1024",
    "note": "Infinity-Cache hits are counted by these memory-side counters"}, indent=1))
