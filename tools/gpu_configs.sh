#!/bin/bash
# Config lines: every BASELINE config in both streams (bench windows, no CPU baseline),
# cfg4 with 1/2/4 replica groups.  Output: gpurun_out/cfgs/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/cfgs"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/lines.txt
for spec in "cfg2 500 50" "run100 1000 50" "cfg4 500 50" "cfg5 300 30"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup $3 --no-cpu-baseline > "$O/bench_$1.json" 2> "$O/bench_$1.err" \
    || { tail -5 "$O/bench_$1.err"; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]); m=d['mt19937']
f=d.get('full_run') or {}; mf=m.get('full_run') or {}
print('$1 philox %.2f us/step %.3g agent-steps/s frac %.3f | full %.2f us/iter || mt19937 %.2f us/step %.3g | full %.2f us/iter %s' % (d['ms_per_step']*1e3, d['value'], d['roofline']['frac'], f.get('seconds',0)/max(1,f.get('iterations',1))*1e6, m['ms_per_step']*1e3, m['value'], mf.get('seconds',0)/max(1,mf.get('iterations',1))*1e6, m['mt_chains']))" | tee -a $O/lines.txt
done
for g in 2 4; do
  timeout -k 10 300 python bench.py --config cfg4 --streams $g --steps 500 --warmup 50 --no-cpu-baseline --no-mt --full-run 0 > "$O/bench_cfg4_s$g.json" 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/bench_cfg4_s$g.json').read().strip().splitlines()[-1]); print('cfg4 philox streams=$g %.2f us/step frac %.3f' % (d['ms_per_step']*1e3, d['roofline']['frac']))" | tee -a $O/lines.txt
done
