#!/bin/bash
# PMC counters of the step kernel by iteration window over iterations 1..N of a fresh cfg3 run
# (one stream: dispatch k = iteration k), one rocprofv3 --pmc pass per counter group, then
# tools/pmc_windows.py.  usage: gpu_pmc_windows.sh [N] [extra window_probe args]
# Output: gpurun_out/pmcw/.
cd "$GRAFT_REPO_ROOT"; N=${1:-600}; shift; O="$GRAFT_REPO_ROOT/gpurun_out/pmcw"; mkdir -p "$O"; export TMPDIR=/tmp
P="$GRAFT_REPO_ROOT/tools/window_probe.py --upto $N --win $N --streams 1 $*"
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $C -d "$O/p$i" -o p$i -- python $P > "$O/p$i.out" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.out"; exit 1; }
done
cd "$GRAFT_REPO_ROOT"
python tools/pmc_windows.py "$O" --win 20 > "$O/windows.txt" && cat "$O/windows.txt"
