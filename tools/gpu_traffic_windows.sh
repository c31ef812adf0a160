#!/bin/bash
# PMC traffic of the step kernel in the bench's windows (the driver's 6-25 and the steady
# 401-600): separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py, the warm-up's
# dispatches skipped -> gpurun_out/tw/traffic_cfg3_w<a>-<b>.json.  usage: gpu_traffic_windows.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/tw"; mkdir -p "$O"; export TMPDIR=/tmp
BA="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-mt --no-steady --full-run 0"
for WK in "5 20" "400 200"; do
  read W K <<< "$WK"; tag="w$((W + 1))-$((W + K))"
  cd /tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc $C -d "$O/$tag/$C" -o p -- python $BA --warmup $W --steps $K > "$O/$tag.$C.out" 2>&1 || { echo "$tag $C failed"; tail -5 "$O/$tag.$C.out"; exit 1; }
  done
  cd "$GRAFT_REPO_ROOT"
  G=$(python -c "import json; print([json.loads(l) for l in open('$O/$tag.FETCH_SIZE.out') if l.startswith('{\"metric')][-1]['config']['streams_per_gpu'])")
  python tools/traffic_json.py "$O/$tag" $((105 * 40000 / G)) cfg3 $G "$((W + 1))-$((W + K))" $((W * G)) > "$O/traffic_cfg3_$tag.json"
  python -c "import json; d=json.load(open('$O/traffic_cfg3_$tag.json')); a=d['agents_per_launch']; print('$tag: %.1f B/agent-step (read %.1f, written %.1f), %s dispatches' % (d['bytes_per_agent_step'], d['fetch_bytes_per_launch']/a, d['write_bytes_per_launch']/a, d['dispatches']))"
done
