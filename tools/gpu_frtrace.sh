#!/bin/bash
# Kernel trace of an MT19937 cfg3 whole run (library-made streams, CU-masked).  Output: gpurun_out/frt/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/frt"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
SPGG_STREAM_MODE=2 SPGG_OWN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/t" -o trace -- \
  python "$GRAFT_REPO_ROOT/tools/fullrun_probe.py" --config cfg3 --rng ${RNG:-mt19937} --iters 1500 > "$O/out.txt" 2>&1 || { tail -5 $O/out.txt; exit 1; }
tail -2 $O/out.txt
