#!/bin/bash
# GPU parity suite, then a longer interleaved cfg3 A/B (5 rounds x 400 iterations) of library builds.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pab; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B cfg3"; timeout -k 10 500 python tools/ab.py --config cfg3 --libs "$@" --steps 400 --rounds 5 2>&1 | grep -v amdgpu.ids | tee $O/ab_cfg3.txt
