#!/bin/bash
# MT19937 whole runs (cfg3, 3000 iterations) by library build x chains per replica, one fresh
# process per run.  usage: gpu_mt_chains_ab.sh "CHAINS..." ROUNDS LIB...
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; CH=$1; R=$2; shift 2
for r in $(seq $R); do for ch in $CH; do for lib in "$@"; do
  v=$(SPGG_LIB="$lib" SPGG_MT_CHAINS=$ch timeout -k 10 120 python tools/fullrun_probe.py --config cfg3 --rng mt19937 --iters 3000 --repeat 2 | tail -1 | sed 's/.*: \([0-9.]*\) us\/iter.*/\1/') || exit 1
  echo "round $r chains $ch $(basename $lib) $v us/iter"
done; done; done
