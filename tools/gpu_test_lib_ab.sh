#!/bin/bash
# Parity suite run against a candidate library (copied over the in-tree one in the box's scratch
# copy only), then a cfg3 A/B (5 rounds x 400 iterations).  usage: gpu_test_lib_ab.sh cand.so ref.so
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pab; mkdir -p $O; export TMPDIR=/tmp
cp "$1" neighbor-aware-reinforcement-learning-fosters-cooperation-in-spatial-public-goods-games-_amd/libspgg_hip.so || exit 1
echo "== pytest gpu ($1)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B cfg3"; timeout -k 10 500 python tools/ab.py --config cfg3 --libs "$2" "$1" --steps 400 --rounds 5 2>&1 | grep -v amdgpu.ids | tee $O/ab_cfg3.txt
