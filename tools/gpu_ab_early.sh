#!/bin/bash
# Early-window A/B of library builds, ONE fresh process per build and round (builds loaded
# into one process share its hardware queues and skew each other): each process runs
# tools/ab.py for one build, 2 rounds (the first pays the code-object load), and the second
# round's us/step and clock are kept.  usage: gpu_ab_early.sh ROUNDS "W K" lib.so...
# Output: gpurun_out/abe/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/abe"; mkdir -p "$O"; export TMPDIR=/tmp
R=$1; read W K <<< "$2"; shift 2
for r in $(seq $R); do
  for L in "$@"; do
    tag=$(basename "$L" .so)
    timeout -k 10 120 python tools/ab.py --config ${CONFIG:-cfg3} --libs "$L" --warmup $W --steps $K --rounds 2 --clock $((K * 50)) > "$O/tmp.txt" 2>&1 || { tail -3 "$O/tmp.txt"; exit 1; }
    grep median "$O/tmp.txt" | sed "s/^/$r /" >> "$O/ab_w${W}_k${K}.txt"
  done
done
python - "$O/ab_w${W}_k${K}.txt" <<'PY'
import re, statistics, sys, collections
d = collections.defaultdict(list); m = collections.defaultdict(list)
for l in open(sys.argv[1]):
    tag = l.split()[1]
    allv = re.search(r"all \[([^\]]*)\]", l).group(1).split(",")
    d[tag].append(float(allv[-1]))
    mm = re.search(r"MHz median (\d+)", l)
    if mm: m[tag].append(float(mm.group(1)))
for t in d:
    print(f"{t:28s} median {statistics.median(d[t]):7.2f} us/step  min {min(d[t]):7.2f}  n={len(d[t])}  MHz {statistics.median(m[t]) if m[t] else 0:.0f}  all {d[t]}")
PY
