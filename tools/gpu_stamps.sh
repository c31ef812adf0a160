#!/bin/bash
# Phase stamps (-DSPGG_STAMPS=1 build, one stream, Philox) of cfg5, cfg3, cfg4, cfg2.  Output: gpurun_out/st/.
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/st"; mkdir -p "$O"; export TMPDIR=/tmp
for c in cfg5 cfg3 cfg4 cfg2; do
  timeout -k 10 200 python tools/stamps.py build_probe/stamps.so --config $c > "$O/phase_stamps_$c.txt" 2>&1 || { tail -5 "$O/phase_stamps_$c.txt"; exit 1; }
  echo "== $c"; grep -v amdgpu.ids "$O/phase_stamps_$c.txt" | head -14
done
