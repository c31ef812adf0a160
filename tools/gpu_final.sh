#!/bin/bash
# Round close-out in one box session: GPU parity suite + smoke, interleaved A/B of library builds
# on cfg3 (args: lib...), then the round evidence of the in-tree library (gpu_round_profile.sh).
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 120 python __graft_entry__.py --smoke > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ $# -gt 0 ]; then
  echo "== A/B cfg3"; timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" --steps 200 --rounds 3 2>&1 | grep -v amdgpu.ids | tee $O/ab_cfg3.txt || exit 1
fi
echo "== round profile"; bash tools/gpu_round_profile.sh
