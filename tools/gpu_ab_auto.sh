#!/bin/bash
# Interleaved A/B of library variants on cfg3 at the default replica grouping and at 1 stream.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/abs; mkdir -p $O; export TMPDIR=/tmp
for s in auto 1; do
  echo "== streams $s"
  if [ $s = auto ]; then unset SPGG_STREAMS; else export SPGG_STREAMS=$s; fi
  timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" --steps 200 --rounds 5 > $O/ab_$s.txt 2>&1; rc=$?
  grep -v amdgpu.ids $O/ab_$s.txt; [ $rc -eq 0 ] || exit $rc
done
