#!/bin/bash
# A/B of run-time settings (environment assignments) on the bench's default window and steady
# window, ONE fresh process per setting and round.  usage: gpu_env_ab.sh ROUNDS "VAR=a" "VAR=b" ...
# ("-" = no assignment).  Output: gpurun_out/envab/ab.txt (one line per run) + a summary.
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/envab"; mkdir -p "$O"; export TMPDIR=/tmp
R=$1; shift
for r in $(seq $R); do
  for E in "$@"; do
    if [ "$E" = "-" ]; then A=(); else A=($E); fi
    timeout -k 10 200 env "${A[@]}" python bench.py --config ${CONFIG:-cfg3} --no-cpu-baseline --no-mt --full-run 0 > "$O/tmp.json" 2> "$O/tmp.err" || { tail -3 "$O/tmp.err"; exit 1; }
    python -c "
import json; d=json.loads(open('$O/tmp.json').read().strip().splitlines()[-1])
print('$r', '$E'.replace(' ', ','), '%.2f %.2f %.2f' % (d['ms_per_step']*1e3, d['roofline']['device_ms_per_step']*1e3, d['steady_window']['ms_per_step']*1e3))" >> "$O/ab.txt"
  done
done
python - "$O/ab.txt" <<'PY'
import collections, statistics, sys
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    p = l.split()
    d[p[1]].append(tuple(map(float, p[2:5])))
for k, v in d.items():
    print(f"{k:40s} window wall {statistics.median(x[0] for x in v):6.2f} device {statistics.median(x[1] for x in v):6.2f} "
          f"steady {statistics.median(x[2] for x in v):6.2f} us/step  n={len(v)}")
PY
