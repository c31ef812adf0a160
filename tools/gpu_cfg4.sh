#!/bin/bash
# cfg4 (8 x L=200, M=2, action state) and cfg5 (L=1000) per-GPU step times, default vs one agent per thread.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for cfg in cfg4 cfg5; do for apt in 0 1; do
  SPGG_APT=$apt timeout -k 10 200 python bench.py --config $cfg --steps 300 --warmup 30 --no-cpu-baseline > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json; exit 1; }
  python -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$cfg apt=$apt', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g'%d['value'])"
done; done
