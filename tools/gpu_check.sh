#!/bin/bash
# Iteration check: the whole GPU parity suite, then bench lines of the given configs
# ("cfg rng steps warmup" specs; default below) and a rocprof kernel summary of the first.
# Output: gpurun_out/check/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/check"; mkdir -p "$O"; export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -4 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
SPECS=${SPECS:-"cfg3:mt19937:200:20 cfg3:philox:300:30 run100:mt19937:1000:50 cfg2:mt19937:500:20"}
first=""
for spec in $SPECS; do
  IFS=: read cfg rng steps warm <<< "$spec"
  [ -z "$first" ] && first="$cfg $rng"
  timeout -k 10 300 python bench.py --config $cfg --rng $rng --steps $steps --warmup $warm --no-cpu-baseline \
    > "$O/bench_${cfg}_${rng}.json" 2> "$O/bench_${cfg}_${rng}.err" || { tail -5 "$O/bench_${cfg}_${rng}.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_${cfg}_${rng}.json').read().strip().splitlines()[-1]); print('$cfg $rng', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g agent-steps/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
set -- $first
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- \
  python "$GRAFT_REPO_ROOT/bench.py" --config $1 --rng $2 --steps 100 --warmup 10 --no-cpu-baseline \
  > "$O/trace.out" 2>&1 || { echo "trace failed"; tail -5 "$O/trace.out"; exit 1; }
find "$O/trace" -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -6
