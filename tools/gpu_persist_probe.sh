#!/bin/bash
# Where a persistent launch's iteration goes (cfg5): phase stamps of the per-launch kernel and of the
# persistent one in timing variants (build_probe/*.so: plain hand-offs, pending record through
# memory), their steady windows, then the MT19937 full run with the barrier-debug build.
# Output: gpurun_out/r6/probe/.
export SPGG_TUNING=1   # SPGG_PERSIST is read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r6/probe; mkdir -p $O; export TMPDIR=/tmp
C=${CFG:-cfg5}
SPGG_PERSIST=0 timeout -k 10 120 python tools/stamps.py build_probe/stamps.so --config $C > $O/st_${C}_perlaunch.txt 2>&1 || exit 1
for v in stamps stamps_plain stamps_norecomp; do
  SPGG_PERSIST=1 timeout -k 10 120 python tools/stamps.py build_probe/$v.so --config $C > $O/st_${C}_$v.txt 2>&1 || exit 1
done
for f in $O/st_${C}_*.txt; do echo "== $f"; grep -v amdgpu.ids $f | head -13; done
: > $O/steady.txt
for v in main plain norecomp; do
  L=$([ $v = main ] && echo "" || echo "build_probe/$v.so")
  SPGG_LIB=$L SPGG_PERSIST=1 timeout -k 10 120 python bench.py --config $C --no-cpu-baseline --no-mt --full-run 0 \
    > $O/bench_$v.json 2> $O/bench_$v.err || { tail -3 $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); s=d['steady_window']
print('$C $v 6-25 %.2f us (dev %.2f) | 401-600 %.2f (dev %.2f)' % (d['ms_per_step']*1e3, d['roofline']['device_ms_per_step']*1e3, s['ms_per_step']*1e3, s['device_ms_per_step']*1e3))" | tee -a $O/steady.txt
done
SPGG_LIB=build_probe/bardebug.so SPGG_PERSIST=1 timeout -k 10 120 python bench.py --config $C --rng mt19937 \
  --no-cpu-baseline --no-steady --full-run 3000 > $O/mt_debug.json 2> $O/mt_debug.err
echo "mt debug rc=$?"; grep -c "spgg barrier" $O/mt_debug.err; grep "spgg barrier" $O/mt_debug.err | head -20
