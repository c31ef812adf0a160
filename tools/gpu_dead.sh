#!/bin/bash
# run() wall time of a sweep-like batch (a third of the replicas absorb early) with and
# without retiring fully-absorbed replica groups.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for skip in 0 1 0 1; do SPGG_SKIP_DEAD=$skip timeout -k 10 200 python - <<'PY' || exit $?
import os, time, sys
sys.path.insert(0, os.getcwd())
import torch, bench
from spgg_amd.engine import BatchEngine
reps = ([bench.runner_params(r=1.0, influence_factor=1.0, seed=s) for s in range(35)] +
        [bench.runner_params(r=3.6, influence_factor=1.0, reward_weight_payoff=1.0, seed=100 + s) for s in range(70)])
eng = BatchEngine(int(os.environ.get("DL", "40")), 3000, reps, use_second_order=False, rng="philox", streams=3)
torch.cuda.synchronize(); t0 = time.perf_counter()
eng.run(snapshots=False)
torch.cuda.synchronize(); dt = time.perf_counter() - t0
st = eng.stopped
print(f"skip_dead={os.environ['SPGG_SKIP_DEAD']} groups={eng.G} live_at_end={[g['live'] for g in eng.groups]} "
      f"absorbed={int((st > 0).sum())} (median stop {int(sorted(st[st > 0])[len(st[st > 0]) // 2]) if (st > 0).any() else 0}) "
      f"run {dt * 1e3:.0f} ms", flush=True)
PY
done
