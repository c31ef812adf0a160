export SPGG_TUNING=1   # the knobs below are read only with the tuning switch
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/fr"; mkdir -p "$O"
for r in 1 2; do
  for E in SPGG_INTERLEAVE=1 SPGG_INTERLEAVE=0; do
    for RNG in philox mt19937; do
      timeout -k 10 200 env $E python tools/fullrun_probe.py --config cfg3 --rng $RNG --iters 10000 > "$O/tmp.txt" 2>&1 || { tail -3 "$O/tmp.txt"; exit 1; }
      echo "$r $E $RNG $(tail -1 $O/tmp.txt)" >> "$O/fr.txt"
    done
  done
done
cat "$O/fr.txt"
