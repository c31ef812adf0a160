#!/bin/bash
# cfg3 throughput by replica count (working-set size) at a fixed number of streams.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/reps; mkdir -p $O; export TMPDIR=/tmp
S=${STREAMS:-3}
for n in ${REPS:-36 54 72 90 105 126 150 210}; do
  timeout -k 10 120 python bench.py --replicas $n --streams $S --no-cpu-baseline --steps 200 > $O/r$n.json 2> $O/r$n.err || exit $?
  python - "$n" "$O/r$n.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
n = int(sys.argv[1])
print(f"reps {n:4d}  state {n*40000*54/1e6:6.0f} MB  {d['ms_per_step']*1e3:7.1f} us/step  {d['value']:.3e} agent-steps/s")
PY
done
