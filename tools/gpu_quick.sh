#!/bin/bash
# quick loop: GPU parity tests + cfg3/cfg2 bench lines (no profiler)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x --no-header -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "$@"; do
  echo "== bench $cfg"; timeout -k 10 300 python bench.py $cfg --no-cpu-baseline | tee -a gpurun_out/bench_quick.jsonl || exit $?
done
