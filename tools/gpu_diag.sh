#!/bin/bash
# Diagnosis pass: ablation A/B timing (build_ablate/*.so), SQ VALU / wave-cycle
# counters of the cfg3 bench, MALL residency probe.  Output: gpurun_out/diag/
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/diag"; mkdir -p "$O"; export TMPDIR=/tmp
echo "== ab"; date
SPGG_STREAMS=6 timeout -k 10 400 python tools/ab.py --config cfg3 --libs "$@" --steps 100 --rounds 4 > "$O/ab.txt" 2>&1 || { tail -20 "$O/ab.txt"; exit 1; }
cat "$O/ab.txt"
cd /tmp
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc $pass -d "$O/pmc$i" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --config cfg3 --no-cpu-baseline --steps 20 --warmup 5 > /dev/null 2> "$O/pmc$i.err" || { echo "pmc $i failed"; tail -5 "$O/pmc$i.err"; }
done
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$O" spgg_step | tee "$O/pmc_summary.txt"
cd "$GRAFT_REPO_ROOT"
echo "== mall"; timeout -k 10 200 python tools/mall_probe.py | tee "$O/mall.txt"
