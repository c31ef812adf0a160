#!/bin/bash
# Persistent launches on the GPU: the persistent-vs-per-launch / oracle tests, then the config lines
# (bench.py per config: window 6-25, steady 401-600, whole run; Philox and MT19937).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r6; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_persistent.py tests/test_gpu_cfg3_deep.py \
  > $O/persist_tests.log 2>&1 || { tail -30 $O/persist_tests.log; exit 1; }
tail -3 $O/persist_tests.log
bash tools/gpu_configs.sh ${@:-cfg2 cfg4 cfg5}
