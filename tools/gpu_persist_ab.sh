#!/bin/bash
# Persistent vs per-launch (SPGG_PERSIST=1 / 0), Philox, bench windows 6-25 and 401-600 + a 3000-iteration
# run, then phase stamps of a persistent launch (-DSPGG_STAMPS=1 build: build_probe/stamps.so).
# Output: gpurun_out/r6/ab/.
export SPGG_TUNING=1   # SPGG_PERSIST is read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6/ab; mkdir -p $O; export TMPDIR=/tmp
: > $O/lines.txt
for c in ${CFGS:-cfg5 cfg4 cfg2}; do
  for p in 1 0; do
    SPGG_PERSIST=$p timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-mt --full-run 3000 \
      > $O/bench_${c}_p$p.json 2> $O/bench_${c}_p$p.err || { tail -5 $O/bench_${c}_p$p.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_${c}_p$p.json').read().strip().splitlines()[-1]); s=d['steady_window']; f=d['full_run']
print('$c persist=$p 6-25 %.2f us (dev %.2f) | 401-600 %.2f (dev %.2f) frac %.3f | 3000-iteration run %.2f us/iter' % (d['ms_per_step']*1e3, d['roofline']['device_ms_per_step']*1e3, s['ms_per_step']*1e3, s['device_ms_per_step']*1e3, s['roofline_frac'], f['seconds']/f['iterations']*1e6))" | tee -a $O/lines.txt
  done
done
for c in ${STAMPS:-cfg5 cfg2}; do
  SPGG_PERSIST=1 timeout -k 10 200 python tools/stamps.py build_probe/stamps.so --config $c --t 30 > $O/stamps_$c.txt 2>&1 \
    || { tail -5 $O/stamps_$c.txt; exit 1; }
  echo "== stamps $c"; grep -v amdgpu.ids $O/stamps_$c.txt | head -16
done
