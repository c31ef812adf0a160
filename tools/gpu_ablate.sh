#!/bin/bash
# Ablation timing (interleaved in-process A/B) + dynamic instruction counts of the step kernel.
#   bash tools/gpu_ablate.sh <config> lib1.so lib2.so ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ablate; export TMPDIR=/tmp
cfg=$1; shift
for s in 6 1; do
  echo "== streams $s"
  SPGG_STREAMS=$s timeout -k 10 300 python tools/ab.py --config $cfg --libs "$@" --steps 100 --rounds 5 || exit $?
done
cd /tmp
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"; do
  tag=${pass%% *}
  timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc $pass -d "$GRAFT_REPO_ROOT/gpurun_out/ablate/$tag" -o p -- python "$GRAFT_REPO_ROOT/bench.py" --config $cfg --no-cpu-baseline --steps 20 --warmup 5 > /dev/null 2> "$GRAFT_REPO_ROOT/gpurun_out/ablate/$tag.err" || { echo "pmc $tag failed"; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/ablate/$tag.err"; exit 1; }
done
python "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/gpurun_out/ablate"
