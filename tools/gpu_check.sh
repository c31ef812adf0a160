#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -x --no-header -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== smoke"; timeout -k 10 120 python __graft_entry__.py --smoke || exit $?
echo "== bench cfg3 philox"; timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-budget 10 | tee gpurun_out/bench_cfg3_philox.json || exit $?
echo "== bench cfg3 mt"; timeout -k 10 300 python bench.py --steps 100 --warmup 20 --rng mt19937 --no-cpu-baseline | tee gpurun_out/bench_cfg3_mt.json || exit $?
echo "== bench cfg2 philox"; timeout -k 10 300 python bench.py --config cfg2 --steps 1000 --warmup 50 --no-cpu-baseline | tee gpurun_out/bench_cfg2.json || exit $?
echo "== rocprof"; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1; echo "rocprof rc=$?"
find "$GRAFT_REPO_ROOT/gpurun_out/prof1" -name "*stats*" | head
