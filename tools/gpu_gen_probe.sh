#!/bin/bash
# MT19937 generator: the MT-stream parity tests, then generator timings of the in-tree and
# build_ablate/ libraries (tools/mt_gen_probe.py).  Output: gpurun_out/gen/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/gen"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 60 --timeout-method thread -p no:cacheprovider \
  -k "${TESTS:-mt or inject or draw or cfg3 or retired}" > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
LIBS="neighbor-aware-reinforcement-learning-fosters-cooperation-in-spatial-public-goods-games-_amd/libspgg_hip.so $(ls build_ablate/*.so 2>/dev/null)"
timeout -k 10 300 python tools/mt_gen_probe.py --libs $LIBS > "$O/probe.txt" 2>&1; rc=$?
grep -v amdgpu.ids "$O/probe.txt"; exit $rc
