#!/bin/bash
# The step kernel's SQ counters with the Philox stream vs with the MT19937 generator running
# beside it (one replica group, so one step launch per iteration; 330 iterations: ~3 generator
# chunks).  Output: gpurun_out/pmcrng/<rng>/<pass>/ and a summary per stream.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/pmcrng"; mkdir -p "$O"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM"
for rng in philox mt19937; do
  extra=$([ $rng = philox ] && echo --no-mt); mkdir -p "$O/$rng"
  for pass in P1 P2; do
    cd /tmp
    timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc ${!pass} -d "$O/$rng/$pass" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --full-run 0 --rng $rng $extra --streams 1 --steps 300 --warmup 30 > "$O/$rng/$pass.out" 2>&1 || { echo "pmc $rng $pass failed"; tail -5 "$O/$rng/$pass.out"; exit 1; }
  done
  cd "$GRAFT_REPO_ROOT"; echo "== $rng step kernel"; python tools/pmc_summary.py "$O/$rng" spgg_step | tee "$O/summary_$rng.txt"
  [ $rng = mt19937 ] && { echo "== mt19937 generator kernel"; python tools/pmc_summary.py "$O/$rng" spgg_mt_gen | tee "$O/summary_gen.txt"; }
done
exit 0
