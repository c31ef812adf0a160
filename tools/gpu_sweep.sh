#!/bin/bash
# usage: gpu_sweep.sh VAR "v1 v2 ..." [bench args...]  -> us/step per value
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  echo -n "$VAR=$v: "
  env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline "$@" | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(f\"{d['ms_per_step']*1e3:.1f} us/step  {d['value']:.3e} agent-steps/s\")" || exit 1
done
