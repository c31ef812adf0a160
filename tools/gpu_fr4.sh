#!/bin/bash
# cfg3 MT19937 whole-run decomposition (2000 iterations, second run, library CU-masked streams):
# both, generator alone (SPGG_TIMING=1), steps alone (=2), recurrence wave priority 0.  Output: gpurun_out/fr4/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fr4"; mkdir -p "$O"; export TMPDIR=/tmp
export SPGG_STREAM_MODE=2 SPGG_OWN_STREAMS=1
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng mt19937 --iters 2000 --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
run both X=1 && run gen_only SPGG_TIMING=1 && run steps_only SPGG_TIMING=2 && run prio0 SPGG_LIB=$(realpath build_ablate/libspgg_prio0.so) \
 && run prio0_gen_only SPGG_TIMING=1 SPGG_LIB=$(realpath build_ablate/libspgg_prio0.so)
