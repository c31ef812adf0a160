#!/bin/bash
# Memory-side traffic of the step kernel split by request size, and the same counters on known-byte
# patterns (tools/traffic_calib.hip) to calibrate them.  One rocprofv3 --pmc pass per counter group
# (at most 2 TCC counters a pass).  Output: gpurun_out/ts/{calib,w6-25,w401-600}/<pass>/ ->
# tools/traffic_split.py.  usage: gpu_traffic_split.sh [windows...]   (default "5 20" "400 200")
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ts"; mkdir -p "$O"; export TMPDIR=/tmp
PASSES=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_64B_sum" "TCC_EA0_RDREQ_128B_sum" "TCC_BUBBLE_sum"
        "TCC_EA0_RDREQ_DRAM_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
run_passes() {  # tag, command...
  local tag=$1; shift; local i=0
  for P in "${PASSES[@]}"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $P -d "$O/$tag/p$i" -o p -- "$@" \
      > "$O/$tag.p$i.out" 2>&1) || { echo "$tag pass $i ($P) failed"; tail -5 "$O/$tag.p$i.out"; return 1; }
  done
}
run_passes calib "$GRAFT_REPO_ROOT/build_probe/traffic_calib" || exit 1
python tools/traffic_split.py calib "$O/calib" > "$O/calib.txt" && cat "$O/calib.txt" || exit 1
WINDOWS=("$@"); [ ${#WINDOWS[@]} -eq 0 ] && WINDOWS=("5 20" "400 200")
for WK in "${WINDOWS[@]}"; do
  read W K <<< "$WK"; tag="w$((W + 1))-$((W + K))"
  run_passes "$tag" python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-mt --no-steady --full-run 0 --warmup $W --steps $K || exit 1
  python tools/traffic_split.py kernel "$O/$tag" $((W * 2)) $((105 * 40000 / 2)) "$((W + 1))-$((W + K))" > "$O/traffic_cfg3_$tag.json" || exit 1
  cat "$O/traffic_cfg3_$tag.json"
done
