#!/bin/bash
# PMC traffic of the step kernel for one source tree (its own built library): separate
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the bench window (cfg3, Philox, the
# auto replica groups) -> gpurun_out/traffic_<tag>/traffic_cfg3.json.
# usage: gpu_traffic.sh TREE_DIR TAG [bench args...]
cd "$GRAFT_REPO_ROOT"; T=$(cd "$1" && pwd); TAG=$2; shift 2
O="$GRAFT_REPO_ROOT/gpurun_out/traffic_$TAG"; mkdir -p "$O"; export TMPDIR=/tmp
BA="$T/bench.py --no-cpu-baseline --no-mt --full-run 0 --steps 40 $*"
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$O/fetch" -o fetch -- python $BA > "$O/fetch.out" 2>&1 || { echo "fetch failed"; tail -5 "$O/fetch.out"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$O/write" -o write -- python $BA > "$O/write.out" 2>&1 || { echo "write failed"; tail -5 "$O/write.out"; exit 1; }
cd "$GRAFT_REPO_ROOT"
G=$(python -c "import json; print([json.loads(l) for l in open('$O/fetch.out') if l.startswith('{\"metric')][-1]['config']['streams_per_gpu'])")
python tools/traffic_json.py "$O" $((105 * 40000 / G)) cfg3 $G > "$O/traffic_cfg3.json"
python -c "import json; d=json.load(open('$O/traffic_cfg3.json')); a=d['agents_per_launch']; print('$TAG: %.1f B/agent-step (read %.1f, written %.1f)' % (d['bytes_per_agent_step'], d['fetch_bytes_per_launch']/a, d['write_bytes_per_launch']/a))"
