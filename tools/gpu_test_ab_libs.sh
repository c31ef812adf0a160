#!/bin/bash
# GPU parity suite (production build), then interleaved A/B of library variants on cfg3
# at 1 and 3 streams (5 rounds each).   usage: gpu_test_ab_libs.sh a.so b.so ...
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tab; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_streams.sh "$@"
