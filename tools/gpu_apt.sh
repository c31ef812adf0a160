#!/bin/bash
# Tilings of the latency-bound configs: agents per thread (SPGG_APT 1 / 2 / max) x replica groups,
# Philox windows (no MT, no whole run), then eager vs hipGraph replay.  Output: gpurun_out/apt/.
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/apt"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/lines.txt
run() {  # name apt streams
  local f="$O/bench_$1_apt$2_s$3.json"
  SPGG_APT=$2 timeout -k 10 200 python bench.py --config $1 --streams $3 --steps 400 --warmup 100 --no-cpu-baseline \
    --no-mt --full-run 0 > "$f" 2> "$f.err" || { tail -5 "$f.err"; exit 1; }
  python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$1 apt=$2 streams=$3 %.2f us/step %.3g agent-steps/s frac %.3f' % (d['ms_per_step']*1e3, d['value'], d['roofline']['frac']))" | tee -a $O/lines.txt
}
for s in 1 2; do for a in max 2; do run cfg4 $a $s; done; done
for a in max 2; do run cfg5 $a 1; done
run cfg5 2 2
for a in 1 2 max; do run cfg2 $a 1; done
for a in 1 2 max; do run run100 $a 1; done
for c in cfg2 run100 cfg4; do
  timeout -k 10 200 python tools/graph_probe.py --config $c --steps 200 --warmup 200 --rounds 3 2>/dev/null | tee -a $O/lines.txt || exit 1
done
