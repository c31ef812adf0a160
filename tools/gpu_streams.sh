#!/bin/bash
# cfg3 step time by number of replica groups (concurrent streams), current library.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for s in 1 2 3 4 5 6; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --streams $s --steps 300 --warmup 30 > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json; exit 1; }
  python -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('streams $s', round(d['ms_per_step']*1e3,2))"
done
for s in 3 2 4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --streams $s --steps 300 --warmup 30 > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json; exit 1; }
  python -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('streams $s', round(d['ms_per_step']*1e3,2))"
done
