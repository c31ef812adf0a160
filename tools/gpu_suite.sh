#!/bin/bash
# The whole GPU test suite (the driver's round-end step) into gpurun_out/r6/pytest_gpu.log.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r6/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r6/pytest_gpu.log; exit $rc
