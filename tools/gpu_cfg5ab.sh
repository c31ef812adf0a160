#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
echo "== cfg5"; timeout -k 10 300 python tools/ab.py --config cfg5 --libs "$@" --steps 300 --warmup 30 --rounds 3 2>&1 | grep -v amdgpu.ids
echo "== cfg4"; timeout -k 10 300 python tools/ab.py --config cfg4 --libs "$@" --steps 300 --warmup 30 --rounds 3 2>&1 | grep -v amdgpu.ids
