#!/bin/bash
# Round evidence (output: gpurun_out/round/):
#   bench.json          default bench line (2 replica groups on concurrent streams, the MT19937 product-path window and whole runs, CPU baseline)
#   trace/              rocprofv3 --kernel-trace --stats of the same command
#   bench_s1.json, trace_s1/   the same with ONE stream (one launch per iteration), so the
#                       kernel's average launch duration equals the per-iteration device time
#   fetch/, write/      --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (separate) -> traffic_cfg3.json
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/round"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail "$O/bench.err"; exit 1; }
cat "$O/bench.json"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-mt --full-run 0 --streams 1 > "$O/bench_s1.json" 2> "$O/bench_s1.err" || { echo "bench s1 failed"; tail "$O/bench_s1.err"; exit 1; }
cat "$O/bench_s1.json"
cd /tmp
BA="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-mt --full-run 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- python $BA > "$O/trace.out" 2>&1 || { echo "trace failed"; tail -5 "$O/trace.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_s1" -o trace -- python $BA --streams 1 > "$O/trace_s1.out" 2>&1 || { echo "trace s1 failed"; tail -5 "$O/trace_s1.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$O/fetch" -o fetch -- python $BA --steps 40 > "$O/fetch.out" 2>&1 || { echo "fetch failed"; tail -5 "$O/fetch.out"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$O/write" -o write -- python $BA --steps 40 > "$O/write.out" 2>&1 || { echo "write failed"; tail -5 "$O/write.out"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python tools/pmc_summary.py "$O" spgg_step > "$O/pmc_summary.txt"; cat "$O/pmc_summary.txt"
G=$(python -c "import json; print(json.load(open('$O/bench.json'))['config']['streams_per_gpu'])")
python tools/traffic_json.py "$O" $((105 * 40000 / G)) cfg3 $G > "$O/traffic_cfg3.json"; cat "$O/traffic_cfg3.json"
for f in trace trace_s1; do echo "== $f"; find "$O/$f" -name "*kernel_stats.csv" -exec cut -c1-220 {} \; ; done
# the MT19937 product path: kernel statistics of its window (step, generator, jump kernels)
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_mt" -o trace -- python "$GRAFT_REPO_ROOT/bench.py" \
  --no-cpu-baseline --rng mt19937 --full-run 0 > "$O/trace_mt.out" 2>&1 || { echo "trace mt failed"; tail -5 "$O/trace_mt.out"; exit 1; }
find "$O/trace_mt" -name "*kernel_stats.csv" -exec cut -c1-220 {} \;
