#!/bin/bash
# Interleaved A/B of library variants on cfg3 at 1 and 3 streams (5 rounds each).
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/abs; mkdir -p $O; export TMPDIR=/tmp
for s in 1 3; do
  echo "== streams $s"; SPGG_STREAMS=$s timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" --steps 200 --rounds 5 > $O/ab_s$s.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/ab_s$s.txt; [ $rc -eq 0 ] || exit $rc
done
