#!/bin/bash
# A/B of two source trees with their own built libraries (e.g. ab_base/ = `git archive HEAD`,
# built there): alternating bench windows, Philox, no CPU baseline / MT / whole run.
# usage: gpu_ab_tree.sh BASE_DIR ROUNDS CONFIG [bench args...]   -> gpurun_out/ab_tree/lines.txt
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ab_tree"; mkdir -p "$O"; export TMPDIR=/tmp
BASE=$1; ROUNDS=$2; CFG=$3; shift 3
for r in $(seq 1 $ROUNDS); do
  for tree in "$BASE" .; do
    tag=$([ "$tree" = . ] && echo new || echo base)
    (cd "$tree" && timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-mt --full-run 0 "$@") \
      > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; exit 1; }
    python -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('round $r $tag $CFG %.2f us/step frac %.3f' % (d['ms_per_step']*1e3, d['roofline']['frac']))" | tee -a $O/lines.txt
  done
done
