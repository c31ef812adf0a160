#!/bin/bash
# MT19937 whole runs (cfg3, 2000 iterations, second run in the process) with library-made group
# streams, per generator build (in-tree: 1 recurrence wave; build_ablate/libspgg_nr2o<k>.so: 2
# recurrence waves, k output waves, <= 32 VGPRs).  MT parity tests per build first.  Output: gpurun_out/fr2/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fr2"; mkdir -p "$O"; export TMPDIR=/tmp
: > $O/fr.txt
for lib in build_ablate/libspgg_nr2o2.so build_ablate/libspgg_nr2o3.so; do
  SPGG_LIB="$(realpath $lib)" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "mt_chained or multi_iteration or mt_stream or equals_host" > "$O/pytest_$(basename $lib).log" 2>&1
  rc=$?; echo "$(basename $lib): $(tail -1 $O/pytest_$(basename $lib).log)"; [ $rc -eq 0 ] || exit $rc
done
for lib in "" build_ablate/libspgg_nr2o2.so build_ablate/libspgg_nr2o3.so; do for mode in 0 2; do
  L=""; [ -n "$lib" ] && L="$(realpath $lib)"
  SPGG_LIB=$L SPGG_STREAM_MODE=$mode SPGG_OWN_STREAMS=1 timeout -k 10 200 python tools/fullrun_probe.py --config cfg3 --rng mt19937 \
    --iters 2000 --repeat 2 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/lib=$(basename ${lib:-in-tree}) mode=$mode /" | tee -a $O/fr.txt || exit 1
done; done
