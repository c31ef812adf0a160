#!/bin/bash
# Cache blocking on/off for batches past the Infinity Cache (cfg3 shape, more replicas),
# then the cache-wave chunk size.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/waves; mkdir -p $O; export TMPDIR=/tmp
run() {  # tag, replicas, env...
  local tag=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --replicas $n --no-cpu-baseline --steps 200 > $O/$tag.json 2> $O/$tag.err || exit $?
  python - "$tag" "$O/$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = d["config"]
print(f"{sys.argv[1]:>14s}  reps {c['replicas_per_gpu']:4d} groups {c['replica_groups']} waves {c['cache_waves']} "
      f"streams {c['streams_per_gpu']}  {d['ms_per_step']*1e3:7.1f} us/step  {d['value']:.3e} agent-steps/s")
PY
}
for n in ${REPS:-105 126 150 210 315 420}; do
  run off_$n $n SPGG_CACHE_MB=100000
  run on_$n $n SPGG_CACHE_MB=240
done
for k in ${CHUNKS:-16 128}; do run chunk${k}_420 420 SPGG_CHUNK=$k; done
