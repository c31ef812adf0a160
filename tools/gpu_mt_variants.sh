#!/bin/bash
# cfg3 in MT19937 mode across generator variants: output waves per chain (build_ablate/
# libspgg_out<k>.so, -DSPGG_GEN_OUT=k; in-tree = 7) x chains per replica.  The MT parity
# tests run first against each variant.  Output: gpurun_out/mtv/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/mtv"; mkdir -p "$O"; export TMPDIR=/tmp
for lib in build_ablate/libspgg_out*.so; do
  SPGG_LIB="$(realpath $lib)" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "mt_chained or multi_iteration or mt_stream or equals_host" > "$O/pytest_$(basename $lib).log" 2>&1
  rc=$?; echo "$(basename $lib): $(tail -1 $O/pytest_$(basename $lib).log)"; [ $rc -eq 0 ] || exit $rc
done
bench() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --full-run 0 --config ${CFG:-cfg3} --rng mt19937 --steps 300 --warmup 30 \
    > "$O/bench_$name.json" 2> "$O/bench_$name.err" || { echo "$name failed"; tail -5 "$O/bench_$name.err"; return 1; }
  python -c "import json; d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step']*1e3,2), 'us/step', '%.3g agent-steps/s'%d['value'], d['config'].get('mt_chains'))"
}
for c in 4 8 16; do bench out7_c$c SPGG_MT_CHAINS=$c || exit 1; done
for o in 3 2; do for c in 4 8 16; do
  bench out${o}_c$c SPGG_LIB="$(realpath build_ablate/libspgg_out$o.so)" SPGG_MT_CHAINS=$c || exit 1
done; done
CFG=cfg5 bench cfg5_out3 SPGG_LIB="$(realpath build_ablate/libspgg_out3.so)" || exit 1
CFG=cfg2 bench cfg2_out3 SPGG_LIB="$(realpath build_ablate/libspgg_out3.so)" || exit 1
