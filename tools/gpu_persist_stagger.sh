#!/bin/bash
# Is the persistent launch's compute slowed by its workgroups leaving the barrier together?  cfg5,
# Philox, steady window 401-600: per-launch, persistent, and persistent with the workgroups' next
# iteration staggered (build_probe/stagger<k>.so: rank (blockIdx/8)%4 sleeps rank x k x ~0.45 us).
export SPGG_TUNING=1
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6/stagger; mkdir -p $O; export TMPDIR=/tmp
C=${CFG:-cfg5}; : > $O/lines.txt
run() {  # name persist lib
  SPGG_LIB=$3 SPGG_PERSIST=$2 timeout -k 10 120 python bench.py --config $C --no-cpu-baseline --no-mt --full-run 0 \
    > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); s=d['steady_window']
print('$C %-12s 6-25 %.2f us (dev %.2f) | 401-600 %.2f (dev %.2f)' % ('$1', d['ms_per_step']*1e3, d['roofline']['device_ms_per_step']*1e3, s['ms_per_step']*1e3, s['device_ms_per_step']*1e3))" | tee -a $O/lines.txt
}
run perlaunch 0 ""
run persist 1 ""
for k in 2 4 8; do run stagger$k 1 build_probe/stagger$k.so; done
run persist_again 1 ""
