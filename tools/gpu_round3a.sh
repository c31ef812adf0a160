#!/bin/bash
# Round-3 check: the GPU suite, the driver's default bench line, and the draw-ring question
# (tools/gpu_fr5.sh).  Output: gpurun_out/r3a/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/r3a"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('philox', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g'%d['value'], 'frac', round(d['roofline']['frac'],3), 'full', round(d['full_run']['seconds']*1e2,2), 'us/iter')
m=d['mt19937']; print('mt', round(m['ms_per_step']*1e3,2), 'us/step', '%.3g'%m['value'], m['mt_chains'], 'full', round(m['full_run']['seconds']*1e2,2), 'us/iter')
print('cpu', '%.3g'%d['cpu_baseline']['value'], d['cpu_baseline'].get('oracle_over_reference'))"
bash tools/gpu_fr5.sh
