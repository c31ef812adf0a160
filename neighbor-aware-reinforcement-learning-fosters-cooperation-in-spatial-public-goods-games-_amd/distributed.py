"""Replica sharding across GPUs: one process per GPU, RCCL only for the final gather.

Replicas (independent (r, kappa, seed, ...) lattices) never exchange data
during a run, so a sweep is sharded as contiguous blocks of the replica list
(the reference's only parallelism is a process pool over experiments,
src/experiments/runner.py:136-154).  At the end every rank all-gathers the
per-replica summaries (final cooperation rate etc.) — one collective of a few
KB-MB over xGMI, latency-bound, never per step.

Works with any torch.distributed backend: "nccl" (RCCL on ROCm) for GPU
tensors, "gloo" for the CPU tests.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch


def local_device() -> Optional[int]:
    """Select this process's GPU before any engine or communicator exists: LOCAL_RANK
    under torchrun (one rank per GPU), else GPU 0.  None without a GPU (CPU / gloo)."""
    if not torch.cuda.is_available():
        return None
    d = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(d)
    return d


def init_from_env(backend: Optional[str] = None) -> bool:
    """Initialise torch.distributed from torchrun's environment (WORLD_SIZE, RANK,
    LOCAL_RANK, MASTER_ADDR/PORT) when WORLD_SIZE > 1 and no group exists yet.

    The GPU is selected first (local_device), so the RCCL communicator binds to this
    rank's device.  backend: $SPGG_DIST_BACKEND, else "nccl" (RCCL on ROCm) with a GPU
    and "gloo" without.  Returns True when this call created the group (the caller
    destroys it)."""
    import torch.distributed as dist
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or dist.is_initialized():
        return False
    backend = backend or os.environ.get("SPGG_DIST_BACKEND")
    dev = local_device()
    if backend is None:
        backend = "nccl" if dev is not None else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    return True


def shard_range(n_items: int, world: int, rank: int):
    """[start, stop) of rank's contiguous block; block sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(items: Sequence, world: int, rank: int):
    a, b = shard_range(len(items), world, rank)
    return list(items[a:b])


def gather_rows(local: np.ndarray, n_items: int, device=None, group=None, dst: Optional[int] = None):
    """Gather each rank's (k_rank, m) float64 block back into (n_items, m), in replica order.

    dst None: all_gather (every rank gets the rows); dst = a rank: gather to that rank only
    (the others get None).  Blocks are padded to the largest shard so a single fixed-size
    collective suffices (no object pickling)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = shard_range(n_items, world, rank)
    local = np.asarray(local, dtype=np.float64)
    if local.ndim == 1:
        local = local[:, None]
    if local.shape[0] != b - a:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, shard is {b - a}")
    m = local.shape[1]
    rows = max(shard_range(n_items, world, r)[1] - shard_range(n_items, world, r)[0] for r in range(world))
    dev = torch.device("cpu") if device is None else torch.device(device)
    buf = torch.zeros((rows, m), dtype=torch.float64, device=dev)
    if b > a:
        buf[: b - a] = torch.from_numpy(local).to(dev)
    if dst is None:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
    else:
        root = dst if group is None else dist.get_global_rank(group, dst)
        parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
        dist.gather(buf, parts, dst=root, group=group)
        if rank != dst:
            return None
    out = np.empty((n_items, m))
    for r in range(world):
        ra, rb_ = shard_range(n_items, world, r)
        out[ra:rb_] = parts[r][: rb_ - ra].cpu().numpy()
    return out


# per replica the final cooperation / defection rates and mean P (the
# return value of the reference's SPGG.run, spgg.py:635-637), the absorbing iteration and the
# iterations run; plus, separately, the cooperation-rate trace (coop_traces)
SUMMARY_FIELDS = ("final_coop", "final_def", "mean_P", "stop_iter", "iterations_run")


def replica_summaries(engine) -> np.ndarray:
    """(R, 5) float64 per-replica summary of a finished BatchEngine.  mean_P is the mean payoff
    of the last iteration a replica started (spgg.py:378, 637): P from S_last, which sits in
    ping-pong buffer (last - 1) & 1 (an absorbed replica's buffers are frozen), so at most two
    payoff launches cover the batch."""
    R = engine.R
    out = np.zeros((R, len(SUMMARY_FIELDS)))
    lasts = [int(engine.last_iteration(k)) for k in range(R)]
    P = {par: engine.payoff_at(par + 1) for par in sorted({(t - 1) & 1 for t in lasts if t >= 1})}
    for k in range(R):
        _, _, S = engine.final_state(k)
        n = S.size
        c = float(np.sum(S == 0)) / n
        mp = float(np.mean(P[(lasts[k] - 1) & 1][k])) if lasts[k] >= 1 else float("nan")
        out[k] = (c, 1.0 - c, mp, float(engine.stopped[k]), float(lasts[k]))
    return out


def coop_traces(engine) -> np.ndarray:
    """(R, iterations) float64 cooperation rate at the start of every iteration (the reference's
    coop_rate_history, spgg.py:383, 595), NaN after a replica's last iteration."""
    st = engine.stats_folded()[:, 1:engine.T + 1, 0].cpu().numpy()   # SPGG_ST_NCOOP, slots 1..T
    out = st / float(engine.L * engine.L)
    lasts = np.array([engine.last_iteration(k) for k in range(engine.R)])
    out[np.arange(engine.T)[None, :] + 1 > lasts[:, None]] = np.nan
    return out


def run_sharded(replicas, L: int, iterations: int, use_second_order=True,
                state_representation="reputation", rng="mt19937", device=None, group=None,
                traces: str = "root"):
    """Run this rank's block of `replicas` on its GPU, then gather the results.

    The rank's GPU is LOCAL_RANK (torchrun) unless `device` names one; replica k of
    the block keeps its global index (shard offset + k) as its Philox stream id, so a
    replica's stream -- and its trajectory in "philox" mode -- does not depend on the
    world size.  Returns (summaries, traces, engine):
      summaries -- (N, 5) float64, SUMMARY_FIELDS, all-gathered to every rank;
      traces    -- (N, iterations) cooperation-rate traces (coop_traces), gathered to rank 0
                   only (traces="root", the default: ~8 B per replica and iteration, which
                   the other ranks rarely need), to every rank ("all"), or not at all
                   ("none"); None on a rank that does not receive them;
      engine    -- this rank's BatchEngine (None for an empty shard).
    These are the path's only collectives."""
    import torch.distributed as dist
    from . import engine as E
    if traces not in ("root", "all", "none"):
        raise ValueError(f"traces must be 'root', 'all' or 'none', not {traces!r}")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if device is None:
        device = local_device()
    elif torch.cuda.is_available():
        torch.cuda.set_device(device)
    a, b = shard_range(len(replicas), world, rank)
    mine = list(replicas[a:b])
    eng = None
    local = np.zeros((0, len(SUMMARY_FIELDS)))
    tr = np.zeros((0, iterations))
    if mine:
        eng = E.BatchEngine(L, iterations, mine, use_second_order=use_second_order,
                            state_representation=state_representation, rng=rng, device=device,
                            replica_offset=a)
        eng.run(snapshots=False)
        local = replica_summaries(eng)
        tr = coop_traces(eng)
    if world == 1:
        return local, (None if traces == "none" else tr), eng
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else None
    summaries = gather_rows(local, len(replicas), device=dev, group=group)
    out_tr = None
    if traces != "none":
        out_tr = gather_rows(tr, len(replicas), device=dev, group=group, dst=0 if traces == "root" else None)
    return summaries, out_tr, eng
