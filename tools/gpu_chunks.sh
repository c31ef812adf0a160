cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/gen
for k in 1 2 8; do
  SPGG_MT_CHUNK=$k timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 60 -p no:cacheprovider -k "equals_host and qlearning" > gpurun_out/gen/chunk$k.log 2>&1
  echo "chunk $k: $(tail -1 gpurun_out/gen/chunk$k.log)"
done
