#!/bin/bash
# Round evidence (output: gpurun_out/round/), all at the driver's window (bench.py defaults:
# iterations 6-25) unless named:
#   bench.json          default bench line (2 replica groups, steady window 401-600, MT19937 window
#                       and whole runs, CPU baseline)
#   trace/              rocprofv3 --kernel-trace --stats of the same window (no MT / steady / full run)
#   bench_s1.json, trace_s1/   the same with ONE stream (one launch per iteration: the kernel's
#                       average launch duration = the per-iteration device time)
#   trace_mt/           kernel statistics of the MT19937 window (step, generator, jump kernels)
#   traffic: tools/gpu_traffic_windows.sh (separate FETCH_SIZE / WRITE_SIZE passes per window)
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/round"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 500 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-mt --no-steady --full-run 0 --streams 1 > "$O/bench_s1.json" 2> "$O/bench_s1.err" || { echo "bench s1 failed"; tail "$O/bench_s1.err"; exit 1; }
cat "$O/bench_s1.json"
cd /tmp
BA="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-mt --no-steady --full-run 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python $BA > "$O/trace.out" 2>&1 || { echo "trace failed"; tail -5 "$O/trace.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_s1" -o trace -- python $BA --streams 1 > "$O/trace_s1.out" 2>&1 || { echo "trace s1 failed"; tail -5 "$O/trace_s1.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_mt" -o trace -- python "$GRAFT_REPO_ROOT/bench.py" \
  --no-cpu-baseline --no-steady --rng mt19937 --full-run 0 > "$O/trace_mt.out" 2>&1 || { echo "trace mt failed"; tail -5 "$O/trace_mt.out"; exit 1; }
cd "$GRAFT_REPO_ROOT"
for f in trace trace_s1 trace_mt; do echo "== $f"; find "$O/$f" -name "*kernel_stats.csv" -exec cut -c1-220 {} \; ; done
bash tools/gpu_traffic_windows.sh
