#!/bin/bash
# cfg3 step time by host enqueue interleaving (SPGG_ENQ_CHUNK; 0 = each group's steps at once).
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/enq; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do for k in ${CHUNKS:-0 2 4 8 16 32}; do
  SPGG_ENQ_CHUNK=$k timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 $EXTRA > $O/k$k.json 2> $O/k$k.err || exit $?
  python -c "import json,sys; d=json.loads(open('$O/k$k.json').read().strip().splitlines()[-1]); print('enq_chunk $k', round(d['ms_per_step']*1e3,1), 'us/step', '%.3e' % d['value'], 'dev', round(d['roofline']['device_ms_per_step']*1e3,1))"
done; done
