#!/bin/bash
# Parity suite run against a candidate library (selected through $SPGG_LIB, so the in-tree
# library is never overwritten), then a cfg3 A/B (5 rounds x 400 iterations).
# usage: gpu_test_lib_ab.sh cand.so ref.so
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pab; mkdir -p $O; export TMPDIR=/tmp
[ -f "$1" ] || { echo "no candidate library $1"; exit 1; }
export SPGG_LIB="$(realpath "$1")"
echo "== pytest gpu ($SPGG_LIB)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
unset SPGG_LIB
echo "== A/B cfg3"; timeout -k 10 500 python tools/ab.py --config cfg3 --libs "$2" "$1" --steps 400 --rounds 5 2>&1 | grep -v amdgpu.ids | tee $O/ab_cfg3.txt
