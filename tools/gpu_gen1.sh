#!/bin/bash
# Single-wave generator: MT parity tests (stop at the first failure), the whole GPU suite, then
# whole-run timings vs the multi-wave generator (SPGG_GEN1=0).  Output: gpurun_out/g1/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/g1"; mkdir -p "$O"; export TMPDIR=/tmp
SPGG_GEN1=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "mt_chained or multi_iteration or mt_stream or equals_host or full_size or cfg3" > "$O/pytest_mt.log" 2>&1
rc=$?; echo "pytest mt: $(tail -1 $O/pytest_mt.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest_mt.log | head -20; exit $rc; }
SPGG_GEN1=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head; exit $rc; }
: > $O/fr.txt
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config ${CFG:-cfg3} --rng ${RNG:-mt19937} --iters ${IT:-2000} --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
run cfg3_gen1 SPGG_GEN1=1 && run cfg3_gen1_only SPGG_TIMING=1 SPGG_GEN1=1 && run cfg3_gen0 SPGG_GEN1=0 && CFG=cfg2 IT=5000 run cfg2_gen1 SPGG_GEN1=1 \
 && CFG=cfg5 IT=1000 run cfg5_gen1 SPGG_GEN1=1 && CFG=run100 IT=10000 run run100_gen1 SPGG_GEN1=1 && CFG=cfg4 IT=3000 run cfg4_gen1 SPGG_GEN1=1 \
 && CFG=cfg4 IT=3000 RNG=philox run cfg4_philox X=1
