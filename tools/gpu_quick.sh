#!/bin/bash
# Quick GPU pass: parity suite, then cfg3 / cfg2 bench lines.  Output: gpurun_out/quick/
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/quick"; mkdir -p "$O"; export TMPDIR=/tmp
echo "== pytest gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -x --no-header -p no:cacheprovider ${PYTEST_ARGS} > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$O/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench cfg3"; timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} | tee "$O/bench_cfg3.json" || exit $?
echo "== bench cfg2"; timeout -k 10 300 python bench.py --config cfg2 --steps 1000 --warmup 50 --no-cpu-baseline | tee "$O/bench_cfg2.json" || exit $?
