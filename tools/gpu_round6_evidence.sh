#!/bin/bash
# Round-6 evidence: the round profile (bench line, rocprof kernel statistics of the driver's window at
# two streams / one stream / MT19937, PMC traffic per window), the available TCC memory-side counters,
# and every single-GPU config's line.  Outputs: gpurun_out/round/, gpurun_out/tw/, gpurun_out/cfgs/.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/round
(cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > "$GRAFT_REPO_ROOT/gpurun_out/round/counters.txt" 2>&1) || true
grep -E "TCC_EA0_(RD|WR)REQ|TCC_BUBBLE|TCC_EA0_RDREQ_(32|64|128)" gpurun_out/round/counters.txt | head -20
bash tools/gpu_round_profile.sh || exit 1
bash tools/gpu_configs.sh cfg2 run100 cfg4 cfg5
