#!/bin/bash
# Step time by iteration window (tools/window_probe.py, iterations 1-600 in 20-iteration windows) of
# library builds, one fresh process per build and round.  usage: gpu_window_lib_ab.sh ROUNDS lib...
# ("base" = the in-tree library).  Output: gpurun_out/wlab/<tag>_r<round>.txt
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/wlab"; mkdir -p "$O"; export TMPDIR=/tmp
R=$1; shift
for r in $(seq 1 $R); do
  for L in "$@"; do
    tag=$(basename "$L" .so); arg=""; [ "$L" = base ] || arg="--lib $GRAFT_REPO_ROOT/$L"
    timeout -k 10 150 python tools/window_probe.py --upto 600 --win 20 $arg > "$O/${tag}_r$r.txt" 2>&1 || { tail -3 "$O/${tag}_r$r.txt"; exit 1; }
  done
done
python - "$O" "$@" <<'PY'
import glob, os, re, statistics, sys
O, libs = sys.argv[1], [os.path.basename(l).replace(".so", "") for l in sys.argv[2:]]
tab = {}
for t in libs:
    for f in sorted(glob.glob(f"{O}/{t}_r*.txt")):
        for l in open(f):
            m = re.match(r"\s*(\d+-\d+)\s+([0-9.]+)", l)
            if m: tab.setdefault(m.group(1), {}).setdefault(t, []).append(float(m.group(2)))
print("window   " + " ".join(f"{t:>12s}" for t in libs) + "   (us/iter, median over rounds)")
for w, d in tab.items():
    print(f"{w:8s} " + " ".join(f"{statistics.median(d.get(t, [0])):12.2f}" for t in libs))
PY
