#!/bin/bash
# GPU parity tests of the in-tree library, then interleaved A/B of library variants on cfg3.
#   bash tools/gpu_parity_ab.sh lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pab; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
[ $# -gt 0 ] || exit 0
echo "== A/B cfg3"; timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" --steps 200 --rounds 3 > $O/ab.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab.txt; exit $rc
