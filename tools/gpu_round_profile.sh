#!/bin/bash
# Round evidence: default bench line (with CPU baseline), rocprofv3 kernel-trace
# stats of the same command, and FETCH_SIZE / WRITE_SIZE passes (separate) for
# the HBM-traffic figure.  Output: gpurun_out/round/
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/round"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
cd /tmp
BA="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python $BA > "$O/trace.out" 2>&1 || { echo "trace failed"; tail -5 "$O/trace.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$O/fetch" -o fetch -- python $BA --steps 40 > "$O/fetch.out" 2>&1 || { echo "fetch failed"; tail -5 "$O/fetch.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$O/write" -o write -- python $BA --steps 40 > "$O/write.out" 2>&1 || { echo "write failed"; tail -5 "$O/write.out"; exit 1; }
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$O" spgg_step > "$O/pmc_summary.txt"; cat "$O/pmc_summary.txt"
cat "$O/trace/trace_kernel_stats.csv" | cut -c1-200
