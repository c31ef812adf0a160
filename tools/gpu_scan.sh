#!/bin/bash
# Where does the step time go?  Ablation A/B, stream-count and replica-count scans,
# FETCH/WRITE traffic of the default cfg3 bench.  Output: gpurun_out/scan/
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/scan"; mkdir -p "$O"; export TMPDIR=/tmp
SPGG_STREAMS=6 timeout -k 10 300 python tools/ab.py --config cfg3 --libs "$@" --steps 100 --rounds 4 > "$O/ab.txt" 2>&1 || { tail -20 "$O/ab.txt"; exit 1; }
cat "$O/ab.txt"
for s in 1 2 3 4 6 8 12; do
  echo -n "streams $s: "; timeout -k 10 120 python bench.py --no-cpu-baseline --streams $s --steps 100 | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['ms_per_step']*1e3,1), 'us/step')" || exit 1
done
for r in 7 14 28 52 105 210 420; do
  echo -n "replicas $r: "; timeout -k 10 120 python bench.py --no-cpu-baseline --replicas $r --steps 100 | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['ms_per_step']*1e3,1), 'us/step', round(d['value']/1e9,2), 'G agent-steps/s', 'streams', d['config']['streams_per_gpu'])" || exit 1
done
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $c -d "$O/$c" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 40 > "$O/$c.out" 2>&1 || { echo "$c failed"; tail -5 "$O/$c.out"; exit 1; }
done
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$O" spgg_step | tee "$O/pmc_summary.txt"
