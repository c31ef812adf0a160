#!/bin/bash
# MT19937 generator layout sweep (chains x iterations per chain) per config.  Output: gpurun_out/mtk/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/mtk"; mkdir -p "$O"; export TMPDIR=/tmp
bench() {  # cfg chains per
  SPGG_MT_CHAINS=$2 SPGG_MT_PER_CHAIN=$3 timeout -k 10 300 python bench.py --no-cpu-baseline --full-run 0 --config $1 \
    --rng mt19937 --steps ${STEPS:-300} --warmup 30 > "$O/bench_$1_c$2_p$3.json" 2> "$O/bench_$1_c$2_p$3.err" \
    || { echo "$1 c$2 p$3 failed"; tail -5 "$O/bench_$1_c$2_p$3.err"; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_$1_c$2_p$3.json').read().strip().splitlines()[-1]); print('$1 c$2 p$3', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g agent-steps/s'%d['value'])"
}
for v in ${SPECS:-"cfg3 16 9" "cfg3 16 4" "cfg3 32 4" "cfg3 32 2" "cfg3 64 2" "cfg3 8 18" "cfg2 32 9" "cfg2 128 9" "run100 8 34" "run100 32 34" "cfg4 32 9" "cfg4 128 4"}; do
  bench $v || exit 1
done
