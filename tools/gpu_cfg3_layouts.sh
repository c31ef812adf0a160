#!/bin/bash
# cfg3 MT19937 whole runs by chain layout (chains x iterations per chain).  Output: gpurun_out/l3/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/l3"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/fr.txt
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng mt19937 --iters 3000 --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
run c8p16 X=1 && run c16p16 SPGG_MT_CHAINS=16 SPGG_MT_PER_CHAIN=16 && run c16p9 SPGG_MT_CHAINS=16 SPGG_MT_PER_CHAIN=9 \
  && run c32p8 SPGG_MT_CHAINS=32 SPGG_MT_PER_CHAIN=8 && run c8p32 SPGG_MT_CHAINS=8 SPGG_MT_PER_CHAIN=32
