#!/bin/bash
# A/B of library builds on bench.py's own windows (the driver's 6-25 and the steady 401-600), ONE
# fresh process per build and round, rounds rotating the order.  Builds: "base" (the in-tree
# library), paths of tuning builds (build_probe/*.so, selected with SPGG_LIB), or env:VAR=VALUE (the
# in-tree library with that tuning knob, under SPGG_TUNING=1).
# usage: gpu_lib_ab.sh ROUNDS lib... [-- bench args]   -> gpurun_out/lab/lines.txt + a median table
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/lab"; mkdir -p "$O"; export TMPDIR=/tmp
R=$1; shift; LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in $(seq 1 $R); do
  n=${#LIBS[@]}
  for i in $(seq 0 $((n - 1))); do
    L=${LIBS[$(( (i + r) % n ))]}
    tag=$(basename "$L" .so); env_lib=""; env_kv=""
    case "$L" in
      base) ;;
      env:*) env_kv="${L#env:}"; tag="$env_kv" ;;   # the in-tree library with a tuning knob set
      *) env_lib="$GRAFT_REPO_ROOT/$L" ;;
    esac
    env SPGG_LIB="$env_lib" ${env_kv:+SPGG_TUNING=1 "$env_kv"} timeout -k 10 180 python bench.py --no-cpu-baseline --no-mt --full-run 0 "$@" > "$O/tmp.json" 2> "$O/tmp.err" \
      || { echo "$tag failed"; tail -5 "$O/tmp.err"; exit 1; }
    python - "$O/tmp.json" "$tag" "$r" >> "$O/lines.txt" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"metric')][-1]
s = d.get("steady_window") or {}
print(f"{sys.argv[3]} {sys.argv[2]} w {d['ms_per_step'] * 1e3:.2f} dev {d['roofline']['device_ms_per_step'] * 1e3:.2f} "
      f"steady {s.get('ms_per_step', 0) * 1e3:.2f} dev {s.get('device_ms_per_step', 0) * 1e3:.2f}")
PY
    tail -1 "$O/lines.txt"
  done
done
python - "$O/lines.txt" <<'PY'
import collections, statistics, sys
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open(sys.argv[1]):
    f = l.split()
    d[f[1]]["w"].append(float(f[3])); d[f[1]]["wd"].append(float(f[5]))
    d[f[1]]["s"].append(float(f[7])); d[f[1]]["sd"].append(float(f[9]))
print("build                      6-25 wall  device | 401-600 wall  device   (medians, n)")
for t, v in d.items():
    m = {k: statistics.median(x) for k, x in v.items()}
    print(f"{t:26s} {m['w']:9.2f} {m['wd']:7.2f} | {m['s']:12.2f} {m['sd']:7.2f}   n={len(v['w'])}")
PY
