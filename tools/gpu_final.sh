#!/bin/bash
# Round-end rehearsal: the GPU suite as the driver runs it, smoke(), the default bench line.
# Output: gpurun_out/final/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/final"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); m=d['mt19937']
print('philox %.2f us/step %.3g frac %.3f full %.2f | mt %.2f us/step full %.2f | cpu %.3g' % (d['ms_per_step']*1e3, d['value'], d['roofline']['frac'], d['full_run']['seconds']*1e2, m['ms_per_step']*1e3, m['full_run']['seconds']*1e2, d['cpu_baseline']['value']))"
