#!/bin/bash
# Whole-run A/B of library builds on the MT19937 product path (and Philox for reference): one
# fresh process per build and round (tools/fullrun_probe.py), rounds rotating the order.
# usage: gpu_mt_lib_ab.sh ROUNDS CONFIG ITERS lib...   (lib: base | path of a tuning build)
#        -> gpurun_out/mtab/lines.txt + medians
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/mtab"; mkdir -p "$O"; export TMPDIR=/tmp
R=$1; CFG=$2; IT=$3; shift 3; LIBS=("$@")
for r in $(seq 1 $R); do
  n=${#LIBS[@]}
  for i in $(seq 0 $((n - 1))); do
    L=${LIBS[$(( (i + r) % n ))]}
    tag=$(basename "$L" .so); env_lib=""
    [ "$L" = base ] || env_lib="$GRAFT_REPO_ROOT/$L"
    for RNG in mt19937 philox; do
      [ "$RNG" = philox ] && [ "$L" != base ] && [ -z "$PHILOX_ALL" ] && continue
      env SPGG_LIB="$env_lib" timeout -k 10 180 python tools/fullrun_probe.py --config $CFG --rng $RNG --iters $IT \
        > "$O/tmp.txt" 2>&1 || { echo "$tag $RNG failed"; tail -5 "$O/tmp.txt"; exit 1; }
      echo "$r $tag $RNG $(tail -1 $O/tmp.txt | sed 's/.*: \([0-9.]*\) us\/iter.*/\1/')" >> "$O/lines.txt"
      tail -1 "$O/lines.txt"
    done
  done
done
python - "$O/lines.txt" <<'PY'
import collections, statistics, sys
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    f = l.split(); d[(f[1], f[2])].append(float(f[3]))
for k, v in sorted(d.items()):
    print(f"{k[0]:12s} {k[1]:8s} median {statistics.median(v):7.2f} us/iter  {v}")
PY
