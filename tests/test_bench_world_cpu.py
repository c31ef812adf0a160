"""bench.py's own multi-rank path (the driver's `torchrun --nproc-per-node N bench.py`), world
size 2 over gloo on CPU, with BatchEngine and the device clock stubbed: each rank times its
own window behind barriers, the agent-steps are summed and the wall time maxed over ranks,
the per-replica cooperation rates and traces are all-gathered, and only rank 0 prints the
JSON line (value = all ranks' agent-steps / the slowest rank's time)."""
import contextlib
import io
import json
import os
import socket
import time

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Event:
    def __init__(self, enable_timing=False):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def _worker(rank, world, port, q):
    import bench
    from spgg_amd import _lib as C
    from spgg_amd import engine as E

    class FakeEngine:
        """BatchEngine's surface as bench.window uses it; rank 1 is the slower rank."""
        made = []

        def __init__(self, L, iterations, replicas, replica_offset=0, **kw):
            self.L, self.T, self.R = L, iterations, len(replicas)
            self.resident = self.G = self.waves = 1
            self.persistent = False
            self.mt_layout = (1, 1)
            self.stop_iter = torch.zeros(self.R, dtype=torch.int32)
            self.st = torch.zeros((self.R, iterations + 2, C.NSTAT), dtype=torch.float64)
            self.t = 1
            FakeEngine.made.append(dict(offset=replica_offset, R=self.R, T=iterations))

        def launch_streams(self):
            return [None]

        def step(self, n, ordered=True):
            time.sleep(0.02 * n * (1 + rank))
            for t in range(self.t, self.t + n):      # a cooperation count per iteration: 100*rank + t
                self.st[:, t + 1, C.ST_NCOOP] = 100 * rank + t
            self.t += n

        def stats_folded(self):
            return self.st

        def check_status(self):
            pass

        def close(self):
            pass

    cur = {"dev": None}
    torch.cuda.set_device = lambda d: cur.__setitem__("dev", int(d))
    torch.cuda.synchronize = lambda *a, **k: None
    torch.cuda.current_stream = lambda *a, **k: None
    torch.cuda.Event = _Event
    E.BatchEngine = FakeEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), SPGG_DIST_BACKEND="gloo")
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        bench.main(["--config", "cfg2", "--steps", "5", "--warmup", "3", "--no-cpu-baseline", "--no-mt", "--no-steady",
                    "--full-run", "0"])
    q.put(dict(rank=rank, stdout=out.getvalue(), dev=cur["dev"], made=FakeEngine.made))


def test_bench_world2_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert outs[1]["stdout"].strip() == ""                 # only rank 0 prints
    line = json.loads(outs[0]["stdout"].strip().splitlines()[-1])
    for o in outs:
        assert o["dev"] == o["rank"]                        # LOCAL_RANK's device
        assert o["made"] == [dict(offset=o["rank"], R=1, T=8)]   # its own replica, global offset
    L, K = 200, 5
    assert line["n_gpus"] == 2 and line["steps"] == K and line["warmup"] == 3
    # value = both ranks' agent-steps / the slower rank's wall time (rank 1: ~2x rank 0's)
    wall_max = line["ms_per_step"] * K / 1e3
    assert abs(line["value"] - 2 * K * L * L / wall_max) <= 1e-9 * line["value"]
    assert wall_max >= 0.02 * K * 2 * 0.9
    # the gather: one row per replica of every rank (final rate + the K-iteration trace)
    g = line["gather"]
    assert g["replicas"] == 2 and g["bytes"] == 2 * (1 + K) * 8
    want = np.mean([(100 * r + 3 + K) / (L * L) for r in range(world)])
    assert abs(g["mean_final_coop"] - want) < 1e-15


def test_rank_seed_blocks_cover_baseline_configs():
    """Ranks split the config's seeds (BASELINE.json configs[3]/[4]): 8 ranks of cfg4 run seeds
    0-63, 8 per rank; 8 ranks of cfg5 run seeds 0-7; every rank keeps the same parameter grid."""
    import bench
    for name, per, total in (("cfg4", 8, 64), ("cfg5", 1, 8), ("cfg2", 1, 8), ("cfg3", 5, 40)):
        seen = []
        for rank in range(8):
            desc, L, M2, state, reps = bench.workload(name, rank)
            seeds = sorted({int(p.seed) for p in reps})
            assert seeds == list(range(per * rank, per * rank + per)), (name, rank, seeds)
            seen += seeds
        assert sorted(seen) == list(range(total)), name
    r0, r1 = bench.workload("cfg3", 0)[4], bench.workload("cfg3", 1)[4]
    assert [(p.r, p.influence_factor) for p in r0] == [(p.r, p.influence_factor) for p in r1]
    assert [p.seed for p in bench.workload("cfg4", 1)[4]] == list(range(8, 16))
    assert bench.seed_range(bench.workload("cfg4", 7)[4]) == "56-63"
