#!/bin/bash
# Quick round check: GPU parity tests, smoke, default bench line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== pytest gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 120 python __graft_entry__.py --smoke || exit $?
echo "== bench"; timeout -k 10 300 python bench.py --steps 300 --warmup 30 --cpu-budget 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
