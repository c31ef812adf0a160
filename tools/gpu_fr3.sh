#!/bin/bash
# MT parity tests, then cfg3 whole-run timings (2000 iterations, second run) MT vs Philox with
# library-made CU-masked streams.  Output: gpurun_out/fr3/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fr3"; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "mt_chained or multi_iteration or mt_stream or equals_host or cfg3" > "$O/pytest.log" 2>&1
rc=$?; echo "pytest: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest.log | head; exit $rc; }
for rng in mt19937 philox; do
  SPGG_STREAM_MODE=${MODE:-2} SPGG_OWN_STREAMS=1 timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng $rng \
    --iters 2000 --repeat 2 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a $O/fr.txt || exit 1
done
for stride in 8 12 16; do for rng in mt19937 philox; do
  SPGG_STREAM_MODE=3 SPGG_GEN_CU_STRIDE=$stride SPGG_OWN_STREAMS=1 timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng $rng \
    --iters 2000 --repeat 2 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/mode3 stride=$stride /" | tee -a $O/fr.txt || exit 1
done; done
