#!/bin/bash
# Replica-group (stream) count A/B on one config's bench line (window 6-25, steady 401-600, whole
# 10,000-iteration run), ONE fresh process per setting and round.  usage: CONFIG=cfg4 gpu_cfg_streams_ab.sh ROUNDS "-" "SPGG_STREAMS=3"
export SPGG_TUNING=1
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/streamsab"; mkdir -p "$O"; export TMPDIR=/tmp
R=$1; shift
for r in $(seq $R); do
  for E in "$@"; do
    if [ "$E" = "-" ]; then A=(); else A=($E); fi
    timeout -k 10 200 env "${A[@]}" python bench.py --config ${CONFIG:-cfg4} --no-cpu-baseline --no-mt > "$O/tmp.json" 2> "$O/tmp.err" || { tail -3 "$O/tmp.err"; exit 1; }
    python -c "
import json; d=json.loads(open('$O/tmp.json').read().strip().splitlines()[-1])
print('$r', '$E'.replace(' ', ','), '%.2f %.2f %.2f %.2f' % (d['ms_per_step']*1e3, d['roofline']['device_ms_per_step']*1e3, d['steady_window']['ms_per_step']*1e3, d['full_run']['seconds']*1e2))" | tee -a "$O/ab.txt"
  done
done
