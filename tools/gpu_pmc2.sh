#!/bin/bash
# Second-level PMC breakdown of the cfg3 step kernel (two passes, counters only).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc2; export TMPDIR=/tmp; cd /tmp
P="rocprofv3 --output-format csv --kernel-trace"
B="python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 300 $P --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc2/a" -o a -- $B > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc2/a.err" || { echo "pass a failed"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/pmc2/a.err"; }
timeout -k 10 300 $P --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_CVT -d "$GRAFT_REPO_ROOT/gpurun_out/pmc2/b" -o b -- $B > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/pmc2/b.err" || { echo "pass b failed"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/pmc2/b.err"; }
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/gpurun_out/pmc2"
