#!/bin/bash
# Ablation / tile-shape timing + rocprofv3 PMC passes on the cfg3 step kernel.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
B="python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 100 --warmup 10"
ms() { python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(f\"{d['ms_per_step']*1e3:.1f} us/step  {d['value']:.3e} agent-steps/s\")"; }
echo "== ablations (cfg3 philox)"
echo -n "full      : "; timeout -k 10 120 $B | ms || exit 1
for m in 1 2 4 7; do echo -n "ablate$m   : "; SPGG_LIB=build_ablate/libspgg_ablate$m.so timeout -k 10 120 $B | ms || exit 1; done
echo "== tile shapes"
for tl in 40x25 50x20 40x20 32x32 64x16 20x20; do echo -n "$tl: "; SPGG_TILE=$tl timeout -k 10 120 $B | ms || exit 1; done
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
cd /tmp
P="rocprofv3 --output-format csv --kernel-trace"
timeout -k 10 300 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/sq" -o sq -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc/sq.err" || { echo "pmc sq failed"; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/pmc/sq.err"; }
timeout -k 10 300 $P --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/fetch" -o fetch -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc/fetch.err" || echo "pmc fetch failed"
timeout -k 10 300 $P --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/write" -o write -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5 > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc/write.err" || echo "pmc write failed"
find "$GRAFT_REPO_ROOT/gpurun_out/pmc" -name "*.csv" | head -20
