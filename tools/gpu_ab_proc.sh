#!/bin/bash
# A/B of library builds over WHOLE runs, one fresh process per run (tools/fullrun_probe.py with
# SPGG_LIB): unlike tools/ab_run.py (all builds in one process) no build inherits another's
# streams or hardware queues.  Rounds rotate the order; each process reports its second run.
# usage: gpu_ab_proc.sh CONFIG RNG ITERS ROUNDS LIB...   -> gpurun_out/ab_proc/<config>_<rng>.txt
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ab_proc"; mkdir -p "$O"; export TMPDIR=/tmp
CFG=$1; RNG=$2; IT=$3; ROUNDS=$4; shift 4
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    v=$(SPGG_LIB="$lib" timeout -k 10 120 python tools/fullrun_probe.py --config $CFG --rng $RNG --iters $IT --repeat 2 | tail -1 | sed 's/.*: \([0-9.]*\) us\/iter.*/\1/') || exit 1
    echo "round $r $CFG $RNG $lib $v us/iter" | tee -a "$O/${CFG}_${RNG}.txt"
  done
done
