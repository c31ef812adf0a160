#!/bin/bash
# Step time by replica-group count at several batch sizes (cfg3 grid cycled), current library.
#   usage: gpu_streams_reps.sh "reps..." "streams..."
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for r in $1; do
  for s in $2; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --replicas $r --streams $s --steps 200 --warmup 20 > /tmp/b.json 2>&1 || { tail -3 /tmp/b.json; exit 1; }
    python -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('reps $r streams $s groups', d['config']['replica_groups'], 'waves', d['config']['cache_waves'], round(d['ms_per_step']*1e3,2), 'us/step', '%.3e' % d['value'])"
  done
done
