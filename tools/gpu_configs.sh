#!/bin/bash
# Per-GPU step time of every single-GPU-sized BASELINE config (in-tree library).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for spec in "cfg2 2000 100" "cfg3 300 30" "cfg4 500 50" "cfg5 300 30"; do
  set -- $spec
  timeout -k 10 200 python bench.py --config $1 --steps $2 --warmup $3 --no-cpu-baseline > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json; exit 1; }
  python -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$1', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g agent-steps/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
