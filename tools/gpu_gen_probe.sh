#!/bin/bash
# MT19937 generator: the MT-stream parity tests (in-tree library, then every build_ablate/
# variant through $SPGG_LIB), then generator timings of all of them (tools/mt_gen_probe.py).
# Output: gpurun_out/gen/.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/gen"; mkdir -p "$O"; export TMPDIR=/tmp
SEL="${TESTS:-multi_iteration or mt_stream or equals_host}"
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 60 --timeout-method thread -p no:cacheprovider \
  -k "$SEL" > "$O/pytest.log" 2>&1
rc=$?; echo "in-tree: $(tail -1 "$O/pytest.log")"; grep -E "^FAILED" "$O/pytest.log" | head -5
for lib in $(ls build_ablate/*.so 2>/dev/null | grep -v _a[0-9]); do
  SPGG_LIB="$(realpath "$lib")" timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 60 \
    --timeout-method thread -p no:cacheprovider -k "$SEL" > "$O/pytest_$(basename "$lib").log" 2>&1
  echo "$(basename "$lib"): $(tail -1 "$O/pytest_$(basename "$lib").log")"
done
LIBS="neighbor-aware-reinforcement-learning-fosters-cooperation-in-spatial-public-goods-games-_amd/libspgg_hip.so $(ls build_ablate/*.so 2>/dev/null)"
timeout -k 10 300 python tools/mt_gen_probe.py --libs $LIBS > "$O/probe.txt" 2>&1; rc=$?
grep -v amdgpu.ids "$O/probe.txt"; exit 0
