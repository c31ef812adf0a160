#!/bin/bash
# Whole-run timing across stream setups (hardware-queue sharing): SPGG_STREAM_MODE (library
# streams: 0 plain, 1 high priority, 2 CU-masked) x SPGG_OWN_STREAMS (group streams from the
# library instead of torch's pool).  Fresh process and after a bench engine.  Output: gpurun_out/fr/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fr"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/fr.txt
for mode in 0 2; do for own in 0 1; do for rng in philox mt19937; do
  SPGG_STREAM_MODE=$mode SPGG_OWN_STREAMS=$own timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng $rng \
    --iters 2000 --repeat 2 2>&1 | grep -v amdgpu.ids | sed "s/^/mode=$mode own=$own /" | tee -a $O/fr.txt || exit 1
  SPGG_STREAM_MODE=$mode SPGG_OWN_STREAMS=$own timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng $rng \
    --iters 2000 --after-bench 2>&1 | grep -v amdgpu.ids | sed "s/^/mode=$mode own=$own /" | tee -a $O/fr.txt || exit 1
done; done; done
