#!/bin/bash
# Dynamic instruction mix of the step kernel (cfg3 bench, default build).  Output: gpurun_out/pmc/
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/pmc"; mkdir -p "$O"; export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$O/avail.txt" 2>&1 || true
grep -o "SQ_INSTS_VALU[A-Z0-9_]*\|SQ_ACTIVE_INST_[A-Z]*\|SQ_INST_CYCLES_[A-Z_]*" "$O/avail.txt" | sort -u > "$O/valu_counters.txt" || true
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VMEM" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc $pass -d "$O/pmc$i" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --config ${CFG:-cfg3} --no-cpu-baseline --steps 20 --warmup 5 > /dev/null 2> "$O/pmc$i.err" || { echo "pmc $i failed"; tail -3 "$O/pmc$i.err"; }
done
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$O" spgg_step | tee "$O/pmc_summary.txt"
cat "$O/valu_counters.txt" | tr '\n' ' '
