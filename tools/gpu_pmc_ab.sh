#!/bin/bash
# PMC passes (one stream: one launch per iteration) for library variants.
#   bash tools/gpu_pmc_ab.sh lib1.so lib2.so ...      output: gpurun_out/pmcab/<lib>/<pass>/
export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/pmcab"; mkdir -p "$O"; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM"
for lib in "$@"; do
  b=$(basename $lib .so)
  mkdir -p "$O/$b"
  for pass in P1 P2; do
    cd /tmp
    SPGG_LIB="$GRAFT_REPO_ROOT/$lib" timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc ${!pass} -d "$O/$b/$pass" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --streams 1 --steps 30 --warmup 5 > "$O/$b/$pass.out" 2>&1 || { echo "pmc $b $pass failed"; tail -5 "$O/$b/$pass.out"; exit 1; }
  done
  cd "$GRAFT_REPO_ROOT"; echo "== $b"; python tools/pmc_summary.py "$O/$b" spgg_step
done
