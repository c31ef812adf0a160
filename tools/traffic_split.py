"""Memory-side traffic by request size from rocprofv3 --pmc passes (tools/gpu_traffic_split.sh).

    python tools/traffic_split.py calib  <dir>                              -> text table
    python tools/traffic_split.py kernel <dir> <skip> <agents> <window>     -> JSON

<dir> holds one sub-directory per pass (p1, p2, ...), each with rocprofv3's counter CSV.  Counters
(TCC block, summed over instances, per dispatch):
  RDREQ, RDREQ_32B, RDREQ_64B, RDREQ_128B   read requests at the L2's memory side, by size
  BUBBLE                                    128-B read requests (FETCH_SIZE's term)
  RDREQ_DRAM_32B                            read requests to DRAM in 32-B units (64 B = 2, 128 B = 4)
  WRREQ, WRREQ_64B                          write requests (WRITE_SIZE = 32 x (WRREQ - 64B) + 64 x 64B)
  WRREQ_WRITE_DRAM_32B                      writes to DRAM in 32-B units
Derived byte counts:
  fetch_size    rocprofv3's FETCH_SIZE expression (BUBBLE x 128 + rest x 64 / x 32)
  read_sized    32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B
  read_dram32   32 x RDREQ_DRAM_32B
  write_size    WRITE_SIZE's expression
  write_dram32  32 x WRREQ_WRITE_DRAM_32B
calib: the known-byte patterns of tools/traffic_calib.hip (in launch order, a flush between each),
each pattern's counts and the following flush's (write-backs of lines the pattern left dirty).
kernel: spgg_step_kernel's dispatches after the first <skip> (the warm-up's), averaged."""
import csv
import glob
import json
import os
import sys

MB = 1 << 20
PATTERNS = [("rd16 stream", 128 * MB), ("rd8 stream", 128 * MB), ("rd4 stream", 128 * MB), ("rd1 stream", 128 * MB),
            ("rd4 48B rows @200B", 32 * MB), ("wr16 stream", 128 * MB), ("wr8 stream", 128 * MB),
            ("wr4 stream", 128 * MB), ("wr1 stream", 128 * MB), ("wr16 half sectors", 128 * MB),
            ("wr16 @64B stride", 32 * MB)]
SHORT = {"TCC_EA0_RDREQ_sum": "RDREQ", "TCC_EA0_RDREQ_32B_sum": "RDREQ_32B", "TCC_EA0_RDREQ_64B_sum": "RDREQ_64B",
         "TCC_EA0_RDREQ_128B_sum": "RDREQ_128B", "TCC_BUBBLE_sum": "BUBBLE",
         "TCC_EA0_RDREQ_DRAM_32B_sum": "RDREQ_DRAM_32B", "TCC_EA0_WRREQ_sum": "WRREQ",
         "TCC_EA0_WRREQ_64B_sum": "WRREQ_64B", "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum": "WRREQ_WRITE_DRAM_32B"}


def load(d):
    """{pass: {(dispatch_id, kernel): {counter: value}}} summed over the CSV's dimension rows."""
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        p = os.path.relpath(f, d).split(os.sep)[0]
        per = out.setdefault(p, {})
        for r in csv.DictReader(open(f)):
            k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            c = SHORT.get(r["Counter_Name"], r["Counter_Name"])
            per.setdefault(k, {})
            per[k][c] = per[k].get(c, 0.0) + float(r["Counter_Value"])
    return out


def derive(c):
    g = lambda k: c.get(k)
    out = {}
    if None not in (g("BUBBLE"), g("RDREQ"), g("RDREQ_32B")):
        out["fetch_size"] = g("BUBBLE") * 128 + (g("RDREQ") - g("BUBBLE") - g("RDREQ_32B")) * 64 + g("RDREQ_32B") * 32
    if None not in (g("RDREQ_32B"), g("RDREQ_64B"), g("RDREQ_128B")):
        out["read_sized"] = 32 * g("RDREQ_32B") + 64 * g("RDREQ_64B") + 128 * g("RDREQ_128B")
    if g("RDREQ_DRAM_32B") is not None:
        out["read_dram32"] = 32 * g("RDREQ_DRAM_32B")
    if None not in (g("WRREQ"), g("WRREQ_64B")):
        out["write_size"] = 32 * (g("WRREQ") - g("WRREQ_64B")) + 64 * g("WRREQ_64B")
    if g("WRREQ_WRITE_DRAM_32B") is not None:
        out["write_dram32"] = 32 * g("WRREQ_WRITE_DRAM_32B")
    return out


def calib(d):
    passes = load(d)
    rows = [dict() for _ in PATTERNS]
    after = [dict() for _ in PATTERNS]
    for p, per in passes.items():
        ids = sorted(per)
        # launch order: flush, (pattern, flush) x len(PATTERNS)
        seq = ids[-2 * len(PATTERNS) - 1:]
        for i in range(len(PATTERNS)):
            rows[i].update(per[seq[1 + 2 * i]])
            after[i].update(per[seq[2 + 2 * i]])
    flush0 = derive(passes[sorted(passes)[0]][sorted(passes[sorted(passes)[0]])[-2 * len(PATTERNS) - 1]])
    cols = ["RDREQ", "RDREQ_32B", "RDREQ_64B", "RDREQ_128B", "BUBBLE", "RDREQ_DRAM_32B", "WRREQ", "WRREQ_64B",
            "WRREQ_WRITE_DRAM_32B"]
    print("# known-byte patterns (tools/traffic_calib.hip); counts per dispatch; bytes as a multiple of the data moved")
    print("%-20s %9s " % ("pattern", "MiB") + " ".join("%11s" % c for c in cols))
    for (name, b), c in zip(PATTERNS, rows):
        print("%-20s %9.0f " % (name, b / MB) + " ".join("%11.0f" % c.get(k, float("nan")) for k in cols))
    print("\n%-20s " % "pattern" + " ".join("%12s" % k for k in
          ("fetch_size", "read_sized", "read_dram32", "write_size", "write_dram32", "+flush wr")))
    for (name, b), c, a in zip(PATTERNS, rows, after):
        dv, da = derive(c), derive(a)
        fl = (da.get("write_size", 0.0) - flush0.get("write_size", 0.0)) / b
        print("%-20s " % name + " ".join("%12.3f" % (dv.get(k, float("nan")) / b) for k in
              ("fetch_size", "read_sized", "read_dram32", "write_size", "write_dram32")) + " %12.3f" % fl)


def kernel(d, skip, agents, window):
    passes = load(d)
    acc, n = {}, {}
    for p, per in passes.items():
        ids = sorted(k for k in per if "spgg_step" in k[1])[skip:]
        for k in ids:
            for c, v in per[k].items():
                acc[c] = acc.get(c, 0.0) + v
                n[c] = n.get(c, 0) + 1
    avg = {c: acc[c] / n[c] for c in acc}
    dv = derive(avg)
    rd, wr = dv["read_sized"] / agents, dv["write_size"] / agents
    print(json.dumps({
        "config": "cfg3", "window": window, "skipped_dispatches": skip, "agents_per_launch": agents,
        "bytes_per_agent_step": rd + wr, "read_bytes_per_agent_step": rd, "write_bytes_per_agent_step": wr,
        "fetch_bytes_per_launch": dv["read_sized"], "write_bytes_per_launch": dv["write_size"],
        "derived_bytes_per_agent_step": {k: v / agents for k, v in dv.items()},
        "counters_per_dispatch": avg, "dispatches": n,
        "method": "rocprofv3 --pmc, one pass per counter group (tools/gpu_traffic_split.sh): reads = 32/64/128 B x "
                  "TCC_EA0_RDREQ_32B/_64B/_128B (no blanket correction: equal to 32 x RDREQ_DRAM_32B), writes = "
                  "WRITE_SIZE's expression; both exact on tools/traffic_calib.hip's known-byte patterns "
                  "(profiles/r06/traffic_calibration.txt)",
        "note": "Infinity-Cache hits are counted by these memory-side counters"}, indent=1))

if __name__ == "__main__":
    if sys.argv[1] == "calib":
        calib(sys.argv[2])
    else:
        kernel(sys.argv[2], int(sys.argv[3]), float(sys.argv[4]), sys.argv[5])
