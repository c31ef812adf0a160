#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_parity_ab.sh "$@" || exit $?
echo "== stamps"; timeout -k 10 300 python tools/stamps.py build_ablate/stamps.so > gpurun_out/stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamps.txt | head -16; exit $rc
