#!/bin/bash
# MT19937 whole runs by generator stream mode (0 plain non-blocking, 2 CU-masked = blocking,
# 4 non-blocking least priority).  Output: gpurun_out/gm/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/gm"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/fr.txt
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config ${CFG:-cfg3} --rng ${RNG:-mt19937} --iters ${IT:-2000} --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
for gm in 0 2 4; do
  run cfg3_g$gm SPGG_GEN_STREAM_MODE=$gm && CFG=cfg4 IT=3000 run cfg4_g$gm SPGG_GEN_STREAM_MODE=$gm \
    && CFG=cfg5 IT=1000 run cfg5_g$gm SPGG_GEN_STREAM_MODE=$gm || exit 1
done
