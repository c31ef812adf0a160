#!/bin/bash
# MT19937 whole runs by generator stream mode (0 non-blocking, 1 non-blocking high priority),
# group streams CU-masked (mode 2).  Output: gpurun_out/r3c/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/r3c"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/fr.txt
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config ${CFG:-cfg3} --rng ${RNG:-mt19937} --iters ${IT:-2000} --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
for gm in 0 1; do
  run cfg3_gen$gm SPGG_GEN_STREAM_MODE=$gm && CFG=cfg2 IT=5000 run cfg2_gen$gm SPGG_GEN_STREAM_MODE=$gm \
   && CFG=cfg5 IT=1000 run cfg5_gen$gm SPGG_GEN_STREAM_MODE=$gm && CFG=run100 IT=10000 run run100_gen$gm SPGG_GEN_STREAM_MODE=$gm || exit 1
done
CFG=run100 IT=10000 RNG=philox run run100_philox X=1
