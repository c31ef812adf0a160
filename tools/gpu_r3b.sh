#!/bin/bash
# GPU suite, then cfg3 whole-run timings: MT19937 (steps + generator, steps alone by ring size),
# Philox.  Output: gpurun_out/r3b/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/r3b"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head; exit $rc; }
: > $O/fr.txt
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python tools/fullrun_probe.py --config ${CFG:-cfg3} --rng ${RNG:-mt19937} --iters ${IT:-2000} --repeat 2 \
  2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/$tag /" | tee -a $O/fr.txt; }
run both X=1 && run steps_default_ring SPGG_TIMING=2 && run steps_ring16 SPGG_TIMING=2 SPGG_MT_CHAINS=1 SPGG_MT_CHUNK=8 \
  && RNG=philox run philox X=1 && CFG=cfg2 IT=5000 run cfg2_mt X=1 && CFG=cfg2 IT=5000 RNG=philox run cfg2_philox X=1 \
  && CFG=cfg5 IT=1000 run cfg5_mt X=1 && CFG=cfg5 IT=1000 RNG=philox run cfg5_philox X=1
