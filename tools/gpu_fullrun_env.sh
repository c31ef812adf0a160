#!/bin/bash
# Whole-run timing (tools/fullrun_probe.py, Philox) of run-time settings, one fresh process each.
# usage: gpu_fullrun_env.sh ROUNDS CONFIG ITERS "VAR=a" ... ("-" = none).  Output: gpurun_out/fre/fr.txt
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fre"; mkdir -p "$O"
R=$1; C=$2; N=$3; shift 3
for r in $(seq $R); do
  for E in "$@"; do
    if [ "$E" = "-" ]; then A=(); else A=($E); fi
    timeout -k 10 200 env "${A[@]}" python tools/fullrun_probe.py --config $C --rng ${RNG:-philox} --iters $N > "$O/tmp.txt" 2>&1 || { tail -3 "$O/tmp.txt"; exit 1; }
    echo "$r $C $E $(tail -1 $O/tmp.txt)" >> "$O/fr.txt"
  done
done
cat "$O/fr.txt"
