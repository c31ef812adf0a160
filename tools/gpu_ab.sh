#!/bin/bash
# A/B timing of library variants on cfg3 (6 streams) and cfg2.  Output: gpurun_out/ab/
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ab"; mkdir -p "$O"; export TMPDIR=/tmp
echo "== cfg3"; timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" > "$O/ab_cfg3.txt" 2>&1; rc=$?; cat "$O/ab_cfg3.txt"; [ $rc -eq 0 ] || exit $rc
echo "== cfg2"; timeout -k 10 400 python tools/ab.py --config cfg2 --libs "$@" --steps 1000 --warmup 50 > "$O/ab_cfg2.txt" 2>&1; rc=$?; cat "$O/ab_cfg2.txt"; [ $rc -eq 0 ] || exit $rc
