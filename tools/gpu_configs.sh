#!/bin/bash
# Config lines: every single-GPU BASELINE config at the bench's default window (iterations 6-25),
# its steady window (401-600) and whole run, Philox and MT19937 (no CPU baseline).
# Output: gpurun_out/cfgs/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/cfgs"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/lines.txt
for c in ${@:-cfg2 run100 cfg4 cfg5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > "$O/bench_$c.json" 2> "$O/bench_$c.err" \
    || { tail -5 "$O/bench_$c.err"; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); m=d['mt19937']; s=d['steady_window']
f=d.get('full_run') or {}; mf=m.get('full_run') or {}
us=lambda r: r.get('seconds',0)/max(1,r.get('iterations',1))*1e6
print('$c philox 6-25 %.2f us/step frac %.3f | 401-600 %.2f frac %.3f | full %.2f us/iter || mt19937 6-25 %.2f | full %.2f us/iter (x%.2f) %s' % (d['ms_per_step']*1e3, d['roofline']['frac'], s['ms_per_step']*1e3, s['roofline_frac'], us(f), m['ms_per_step']*1e3, us(mf), us(mf)/max(us(f),1e-9), m['mt_chains']))" | tee -a $O/lines.txt
done
