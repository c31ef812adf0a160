#!/bin/bash
# cfg2 (one L=200 replica): wall vs kernel time per step (host-launch bound?)
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/cfg2"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --config cfg2 --steps 2000 --warmup 100 --no-cpu-baseline > $O/bench.json 2>&1 || exit 1
tail -1 $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python "$GRAFT_REPO_ROOT/bench.py" --config cfg2 --steps 2000 --warmup 100 --no-cpu-baseline > "$O/trace.out" 2>&1 || exit 1
find "$O/trace" -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -4
