#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for alg in double_qlearning qlearning; do
  SPGG_GEN1=1 timeout -k 10 120 python tools/debug_gen1.py $alg 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
  SPGG_GEN1=0 timeout -k 10 120 python tools/debug_gen1.py $alg 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
  python tools/debug_gen1.py $alg compare
done
