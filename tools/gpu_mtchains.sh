#!/bin/bash
# MT19937 chained generator: the MT parity tests first (stop at the first failure), the whole
# GPU suite, then MT19937 bench lines of every config (auto chains) and cfg3 chain variants.
# Output: gpurun_out/mtc/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/mtc"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "mt_chained or multi_iteration or mt_stream or equals_host or full_size" > "$O/pytest_mt.log" 2>&1
rc=$?; tail -3 "$O/pytest_mt.log"; [ $rc -eq 0 ] || { grep -E "^E |Error" "$O/pytest_mt.log" | head -20; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || { grep -E "^E |Error" "$O/pytest_gpu.log" | head -20; exit $rc; }
bench() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --full-run 0 $BARGS > "$O/bench_$name.json" 2> "$O/bench_$name.err" \
    || { echo "$name failed"; tail -5 "$O/bench_$name.err"; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g agent-steps/s'%d['value'], d['config'].get('mt_chains'))"
}
for cfg in cfg3 cfg2 run100 cfg4 cfg5; do
  BARGS="--config $cfg --rng mt19937 --steps 300 --warmup 30" bench ${cfg}_auto SPGG_X=1 || exit 1
done
for v in "1 8" "2 4" "2 9" "4 4" "4 9"; do
  set -- $v
  BARGS="--config cfg3 --rng mt19937 --steps 300 --warmup 30" bench cfg3_c$1_p$2 SPGG_MT_CHAINS=$1 SPGG_MT_PER_CHAIN=$2 || exit 1
done
