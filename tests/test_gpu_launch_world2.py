"""bench.py's multi-rank launch path on the GPU box: `torchrun --nproc-per-node 2 bench.py`, both
ranks on the box's one MI355X (gloo collectives: RCCL refuses two ranks on one device).  Each
rank steps its own shard of real replicas through the HIP kernels (seeds offset by rank, global
Philox stream ids), the windows are timed behind barriers, the agent-steps summed and the wall
time maxed over ranks, and the per-replica cooperation rates and traces all-gathered; rank 0
prints the one JSON line.  The reference fans replicas out over a process pool
(src/experiments/runner.py:136-154); the 8-GPU node runs the same path with RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_on_one_gpu():
    env = dict(os.environ, SPGG_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--config", "cfg4", "--steps", "20", "--warmup", "5", "--no-cpu-baseline",
           "--no-mt", "--full-run", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 20 and d["value"] > 0
    assert d["config"]["replicas_per_gpu"] == 8
    g = d["gather"]
    assert g["replicas"] == 16 and g["bytes"] == 16 * (1 + 20) * 8   # final rate + 20-step trace, f64
    assert 0.0 < g["mean_final_coop"] < 1.0
