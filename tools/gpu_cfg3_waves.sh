#!/bin/bash
# cfg3 (105 replicas) under different group / cache-wave splits.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/cfg3w; mkdir -p $O; export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 > $O/$tag.json 2> $O/$tag.err || exit $?
  python - "$tag" "$O/$tag.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
c = d["config"]
print(f"{sys.argv[1]:>12s} groups {c['replica_groups']} waves {c['cache_waves']} streams {c['streams_per_gpu']}  "
      f"{d['ms_per_step']*1e3:7.1f} us/step  {d['value']:.3e}")
PY
}
for rep in 1 2; do
run default_$rep
run c120_$rep SPGG_CACHE_MB=120
run c120s6_$rep SPGG_CACHE_MB=120 SPGG_STREAMS=6
run c80s6_$rep SPGG_CACHE_MB=80 SPGG_STREAMS=6
run c60s8_$rep SPGG_CACHE_MB=60 SPGG_STREAMS=8
run s6_$rep SPGG_STREAMS=6
done
