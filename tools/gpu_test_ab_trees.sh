#!/bin/bash
# GPU parity suite of this tree, then tools/gpu_ab_trees.sh <tree_a> <tree_b> [rounds].
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tab; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_trees.sh "$@"
