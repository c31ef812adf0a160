#!/bin/bash
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pab; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B cfg2"; timeout -k 10 300 python tools/ab.py --config cfg2 --libs "$@" --steps 2000 --warmup 100 --rounds 3 2>&1 | grep -v amdgpu.ids
echo "== A/B cfg3"; timeout -k 10 300 python tools/ab.py --config cfg3 --libs "$@" --steps 200 --rounds 3 2>&1 | grep -v amdgpu.ids
