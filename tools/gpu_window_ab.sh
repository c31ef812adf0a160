#!/bin/bash
# Early (iterations 1-100) and steady (401-460) step time and effective clock
# (tools/window_probe.py --clock) of several library builds, one fresh process each.
# usage: gpu_window_ab.sh lib.so... (paths relative to the repo; "base" = the in-tree library)
# Output: gpurun_out/wab/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/wab"; mkdir -p "$O"; export TMPDIR=/tmp
for L in "$@"; do
  tag=$(basename "$L" .so); arg=""; [ "$L" = base ] || arg="--lib $GRAFT_REPO_ROOT/$L"
  timeout -k 10 120 python tools/window_probe.py --upto 100 --win 20 --clock 900 $arg > "$O/early_$tag.txt" 2>&1 || { tail -3 "$O/early_$tag.txt"; exit 1; }
  timeout -k 10 120 python tools/window_probe.py --first 400 --upto 60 --win 20 --clock 900 $arg > "$O/steady_$tag.txt" 2>&1 || { tail -3 "$O/steady_$tag.txt"; exit 1; }
  echo "== $tag"; grep -E "^ *[0-9]+-" "$O/early_$tag.txt" | tail -4; grep -E "^ *[0-9]+-" "$O/steady_$tag.txt"
done
