"""The multi-GPU launch path, world size 2 over gloo on CPU, with the GPU work stubbed:
`sweep.main` under torchrun's environment, `sweep.run_experiments`' distributed branch
and `distributed.run_sharded` (the replacement of the reference's process-pool fan-out,
src/experiments/runner.py:136-154).  Checks that each rank runs exactly its own
contiguous block, on the GPU named by LOCAL_RANK, with global Philox stream ids, and
that every rank gets the full result list in input order."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_coop(p):
    return round(p[0] * 0.1 + p[1] * 0.01 + (0.001 if p[2] else 0.0), 6)


class _FakeEngine:
    """Stands in for BatchEngine: records how it was built, no GPU work."""
    made = []

    def __init__(self, L, iterations, replicas, device=None, replica_offset=0, **kw):
        self.L, self.T, self.reps = L, iterations, list(replicas)
        self.R = len(self.reps)
        self.stopped = np.zeros(self.R, dtype=np.int64)
        _FakeEngine.made.append(dict(seeds=[p.seed for p in self.reps], device=device,
                                     offset=replica_offset, cur_dev=torch.cuda.current_device()))

    def run(self, **kw):
        pass

    def final_state(self, k):
        S = np.ones((self.L, self.L), dtype=np.int64)
        S.flat[: int(self.reps[k].seed) % (self.L * self.L)] = 0    # coop count = seed
        return None, None, S

    def last_iteration(self, k):
        return self.T

    def payoff_at(self, t):                          # P = seed / 100 everywhere, from S_t's buffer
        return np.stack([np.full((self.L, self.L), p.seed / 100.0) for p in self.reps])

    def stats_folded(self):                          # NCOOP of slot t = seed + t
        st = torch.zeros((self.R, self.T + 2, 34), dtype=torch.float64)
        for k, p in enumerate(self.reps):
            st[k, :, 0] = torch.arange(self.T + 2, dtype=torch.float64) + p.seed
        return st


def _worker(rank, world, ports, q):
    import spgg_amd  # noqa: F401
    from spgg_amd import distributed as D
    from spgg_amd import engine as E
    from spgg_amd import sweep as SW
    from spgg_amd.engine import ReplicaParams

    # a "GPU" per rank: device selection is recorded, no device is touched
    cur = {"dev": None}
    torch.cuda.is_available = lambda: True
    torch.cuda.set_device = lambda d: cur.__setitem__("dev", int(d))
    torch.cuda.current_device = lambda: cur["dev"]
    ran = []

    def fake_run_batch(params, seeds=None, device=None, save_png=True, verbose=True, progress=None, **kw):
        ran.append(dict(params=list(params), seeds=list(seeds or []), device=device, cur_dev=cur["dev"]))
        return [(p, (_fake_coop(p), 0)) for p in params]

    SW.run_batch = fake_run_batch
    E.BatchEngine = _FakeEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", LOCAL_RANK=str(rank), SPGG_DIST_BACKEND="gloo")
    out = {"rank": rank}

    # 1. an already-initialised group: run_experiments' distributed branch and run_sharded
    os.environ["MASTER_PORT"] = str(ports[0])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        combos = [(r, k, so, 0.8, 1.0, 1.0, "reputation", "qlearning")
                  for r in (2.0, 3.0, 4.0) for k in (0.0, 1.0) for so in (False, True)][:11]
        res = SW.run_experiments(combos, use_progress_bar=False, seeds=list(range(100, 111)))
        out["rx_results"] = [(p, c) for p, (c, _) in res]
        out["rx_ran"] = ran[:]
        reps = [ReplicaParams(r=3.0, seed=s) for s in range(5, 12)]    # 7 replicas
        summ, traces, eng = D.run_sharded(reps, L=4, iterations=9, rng="philox")
        out["sharded"] = summ
        out["traces"] = traces
        summ2, traces_all, _ = D.run_sharded(reps, L=4, iterations=9, rng="philox", traces="all")
        out["traces_all"] = traces_all
        out["sharded2"] = summ2
        out["engine"] = _FakeEngine.made[-1]
    finally:
        dist.destroy_process_group()

    # 2. sweep.main under torchrun's environment initialises (and destroys) its own group
    ran.clear()
    os.environ.update(MASTER_PORT=str(ports[1]), WORLD_SIZE=str(world), RANK=str(rank))
    res = SW.main(["--experiment-type", "figure_6_7_8_9", "--no-progress"])
    out["main_results"] = [(p, c) for p, (c, _) in res]
    out["main_ran"] = ran[:]
    out["main_destroyed"] = not dist.is_initialized()
    q.put(out)


def test_launch_path_world2_gloo():
    world = 2
    ports = (_free_port(), _free_port())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, ports, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    from spgg_amd.distributed import shard_range
    from spgg_amd import sweep as SW

    # run_experiments: disjoint contiguous blocks, each on its rank's device, gathered in order
    combos = [(r, k, so, 0.8, 1.0, 1.0, "reputation", "qlearning")
              for r in (2.0, 3.0, 4.0) for k in (0.0, 1.0) for so in (False, True)][:11]
    for o in outs:
        a, b = shard_range(len(combos), world, o["rank"])
        assert len(o["rx_ran"]) == 1
        call = o["rx_ran"][0]
        assert call["params"] == combos[a:b]                 # its own tuples, nobody else's
        assert call["seeds"] == list(range(100 + a, 100 + b))
        assert call["device"] == o["rank"] and call["cur_dev"] == o["rank"]
        assert [p for p, _ in o["rx_results"]] == combos     # every rank: the full list, input order
        assert [c for _, c in o["rx_results"]] == [_fake_coop(p) for p in combos]

    # run_sharded: shard offset = global replica index base (Philox stream ids), device per rank
    for o in outs:
        a, b = shard_range(7, world, o["rank"])
        e = o["engine"]
        assert e["seeds"] == list(range(5 + a, 5 + b)) and e["offset"] == a
        assert e["device"] == o["rank"] and e["cur_dev"] == o["rank"]
        want = np.array([[s / 16, 1 - s / 16, s / 100, 0.0, 9.0] for s in range(5, 12)])
        np.testing.assert_allclose(o["sharded"], want)
        # the cooperation-rate traces of every replica, gathered in replica order: to rank 0
        # only by default, to every rank with traces="all"
        want_tr = [[(s + t) / 16 for t in range(1, 10)] for s in range(5, 12)]
        if o["rank"] == 0:
            np.testing.assert_allclose(o["traces"], want_tr)
        else:
            assert o["traces"] is None
        np.testing.assert_allclose(o["traces_all"], want_tr)
        np.testing.assert_allclose(o["sharded2"], want)

    # sweep.main under torchrun env: each rank runs its block only, results complete
    cfg = SW.load_config(None)
    all_combos = [(*p, "qlearning") for p in SW.generate_param_combinations(cfg, "figure_6_7_8_9")]
    ran = []
    for o in outs:
        assert o["main_destroyed"]
        a, b = shard_range(len(all_combos), world, o["rank"])
        assert [c["params"] for c in o["main_ran"]] == [all_combos[a:b]]
        assert o["main_ran"][0]["device"] == o["rank"]
        ran += o["main_ran"][0]["params"]
        assert [p for p, _ in o["main_results"]] == all_combos
    assert ran == all_combos
