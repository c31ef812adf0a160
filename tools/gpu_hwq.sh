#!/bin/bash
# cfg3 step time by HIP hardware queues per process (GPU_MAX_HW_QUEUES) and replica groups.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/hwq; mkdir -p $O; export TMPDIR=/tmp
for q in ${QUEUES:-4 8 16}; do for s in ${STREAMS:-3 4 6 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --streams $s > $O/q${q}s$s.json 2> $O/q${q}s$s.err || exit $?
  python -c "import json,sys; d=json.loads(open('$O/q${q}s$s.json').read().strip().splitlines()[-1]); print('hwq $q streams $s', round(d['ms_per_step']*1e3,1), 'us/step', '%.3e' % d['value'])"
done; done
