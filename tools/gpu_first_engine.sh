#!/bin/bash
# First-engine window probe (tools/first_engine_probe.py): ROUNDS rounds of one fresh process per
# mode.  Output: gpurun_out/first/probe.txt + medians.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/first"; mkdir -p "$O"; export TMPDIR=/tmp
R=${1:-3}; shift; MODES=${@:-none busy engine alloc streams}
for r in $(seq $R); do
  for m in $MODES; do
    timeout -k 10 120 python tools/first_engine_probe.py $m 2> "$O/err.txt" | sed "s/^/$r /" >> "$O/probe.txt" || { tail -5 "$O/err.txt"; exit 1; }
  done
done
python - "$O/probe.txt" <<'PY'
import collections, statistics, sys
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split(); d[p[1]].append(float(p[2]))
for k, v in d.items():
    print(f"{k:10s} median {statistics.median(v):7.2f} min {min(v):7.2f} max {max(v):7.2f} n={len(v)}")
PY
