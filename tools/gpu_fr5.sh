#!/bin/bash
# cfg3 MT19937 step kernels alone (SPGG_TIMING=2) by draw-ring size (chunk = chains x per_chain,
# ring = 2 chunks), and Philox.  Output: gpurun_out/fr5/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fr5"; mkdir -p "$O"; export TMPDIR=/tmp
export SPGG_STREAM_MODE=2 SPGG_OWN_STREAMS=1
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng ${RNG:-mt19937} --iters 2000 --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
run steps_c1_k8 SPGG_TIMING=2 SPGG_MT_CHAINS=1 SPGG_MT_CHUNK=8 && run steps_c16_p2 SPGG_TIMING=2 SPGG_MT_CHAINS=16 SPGG_MT_PER_CHAIN=2 \
 && run steps_c16_p9 SPGG_TIMING=2 && run both_c16_p2 SPGG_MT_CHAINS=16 SPGG_MT_PER_CHAIN=2 && RNG=philox run philox X=1
