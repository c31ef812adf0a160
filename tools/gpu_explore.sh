#!/bin/bash
# Exploration: variant libraries (A/B) and stream / replica-count sweeps on cfg3.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/explore; mkdir -p $O; export TMPDIR=/tmp
echo "== A/B variants"; timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" --steps 200 --rounds 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
for s in 1 2 3 4 6; do
  echo "== streams $s"; timeout -k 10 120 python bench.py --no-cpu-baseline --streams $s --steps 200 > $O/s$s.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('$O/s$s.json'));print(d['ms_per_step']*1e3, d['roofline']['frac'])"
done
for r in 210 420; do
  echo "== replicas $r"; timeout -k 10 120 python bench.py --no-cpu-baseline --replicas $r --steps 100 > $O/r$r.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('$O/r$r.json'));print(d['ms_per_step']*1e3, d['value'], d['config']['streams_per_gpu'])"
done
