#!/bin/bash
# Round-3 starting point: step time of every config in both random streams, and the
# rocprof kernel statistics of the MT19937 path (output: gpurun_out/r3base/).
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/r3base"; mkdir -p "$O"; export TMPDIR=/tmp
for spec in "cfg3 philox 300 30" "cfg3 mt19937 100 20" "cfg2 philox 1000 50" "cfg2 mt19937 300 20" \
            "run100 mt19937 500 20" "run100 philox 1000 50" "cfg4 philox 500 50" "cfg4 mt19937 100 20" \
            "cfg5 philox 300 30" "cfg5 mt19937 30 5"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --rng $2 --steps $3 --warmup $4 --no-cpu-baseline \
    > "$O/bench_$1_$2.json" 2> "$O/bench_$1_$2.err" || { tail -5 "$O/bench_$1_$2.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$1_$2.json').read().strip().splitlines()[-1]); print('$1 $2', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g agent-steps/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_mt" -o trace -- \
  python "$GRAFT_REPO_ROOT/bench.py" --rng mt19937 --steps 40 --warmup 5 --no-cpu-baseline > "$O/trace_mt.out" 2>&1 \
  || { echo "trace failed"; tail -5 "$O/trace_mt.out"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_run100" -o trace -- \
  python "$GRAFT_REPO_ROOT/bench.py" --config run100 --rng mt19937 --steps 200 --warmup 5 --no-cpu-baseline \
  > "$O/trace_run100.out" 2>&1 || { echo "trace failed"; tail -5 "$O/trace_run100.out"; exit 1; }
for f in trace_mt trace_run100; do echo "== $f"; find "$O/$f" -name "*kernel_stats.csv" -exec cut -c1-200 {} \; ; done
