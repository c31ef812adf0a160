"""Benchmark: SPGG hot path on MI355X, agent-steps/s (+ roofline, CPU baseline).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3] [--rng philox]

Default window: the driver's, iterations 6-25 (--warmup 5 --steps 20); the line also carries
the steady window 401-600 (eps at eps_min), the whole 10,000-iteration run (full_run) and the
MT19937 product path (mt19937).

A "step" is one iteration of the reference's run loop (src/model/spgg.py:368-592)
over every replica of the batch resident in HBM.  Default workload is cfg3 of
BASELINE.json (L=200, r in {2.0..5.0} x kappa in {0,0.5,1.0} x 5 seeds = 105
replicas, M=1, reputation state, w_P=1.0) — the L=200 single-GPU configuration
the metric and its roofline target are quoted on.  Under torchrun each rank runs
its own block of the config's seeds (cfg4: seeds 8k..8k+7 on rank k, so 8 ranks run
BASELINE's seeds 0-63; weak scaling); the only collective is the
final cooperation-rate gather (RCCL all_gather).

value = executed agent-steps of all ranks / max-over-ranks wall time of the K
timed steps (absorbed replicas stop contributing, as in the reference).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-steps/sec (L×L×iters×replicas) + achieved HBM GB/s, L=200"
ALGO_BYTES_PER_AGENT_STEP = 58.0   # S 1+1, R 8+8, Q 32 read + 8 written
HBM_PEAK_GBS = 8000.0              # MI355X HBM3E peak (MI355X_MICROARCH.md)


def runner_params(**kw):
    from spgg_amd.engine import ReplicaParams
    base = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99,
                epsilon_min=0.01, lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10,
                rep_gain_C=1.0, reward_weight_payoff=0.95, influence_factor=1.0, r=3.0)
    base.update(kw)
    return ReplicaParams(**base)


def workload(name, rank):
    """(description, L, M2, state, [ReplicaParams]) of a BASELINE.json config for one rank.

    Ranks split the config's seeds (BASELINE.json configs[3]/[4]: cfg4 = seeds 0-63, 8 per GPU;
    cfg5 = seeds 0-7, one per GPU): rank k runs seeds k*S .. k*S+S-1, S = the config's seeds per
    GPU, so N ranks together run seeds 0 .. N*S-1 -- the reference runner's replica set
    (runner.py:136-154 fans the same replicas out over a process pool)."""
    if name == "cfg2":
        off = rank
        return ("cfg2: L=200 r=3.0 kappa=1.0 M=1 reputation, 1 replica", 200, False, "reputation",
                [runner_params(r=3.0, influence_factor=1.0, seed=off)])
    if name == "cfg3":  # the r x kappa grid, 5 seeds per GPU
        off = 5 * rank
        reps = [runner_params(r=2.0 + 0.5 * i, influence_factor=k, reward_weight_payoff=1.0, seed=off + s)
                for i in range(7) for k in (0.0, 0.5, 1.0) for s in range(5)]
        return ("cfg3: L=200 r{2.0..5.0}x kappa{0,0.5,1}x5 seeds = 105 replicas, M=1 reputation, w_P=1.0",
                200, False, "reputation", reps)
    if name == "cfg4":
        off = 8 * rank
        return ("cfg4: L=200 r=3.0 kappa=1.0 M=2 action, 8 replicas per GPU", 200, True, "action",
                [runner_params(r=3.0, influence_factor=1.0, seed=off + s) for s in range(8)])
    if name == "cfg5":
        off = rank
        return ("cfg5: L=1000 r=3.6 kappa=1.0 M=1 reputation, 1 replica per GPU", 1000, False, "reputation",
                [runner_params(r=3.6, influence_factor=1.0, seed=off)])
    if name == "run100":  # the shape one SPGG(...).run() of the reference's runner steps (runner.py:88-101)
        off = rank
        return ("run100: L=100 r=3.0 kappa=1.0 M=1 reputation, 1 replica (one SPGG.run of the runner)", 100,
                False, "reputation", [runner_params(r=3.0, influence_factor=1.0, seed=off)])
    raise SystemExit(f"unknown config {name}")


def seed_range(reps):
    """'a-b' (or 'a') of a rank's replica seeds, for the line's config."""
    s = sorted({int(p.seed or 0) for p in reps})
    return f"{s[0]}-{s[-1]}" if len(s) > 1 else f"{s[0]}"


def latest_profile(name):
    """The newest round's copy of a measured file under profiles/r<NN>/ (None if absent)."""
    pdir = os.path.join(ROOT, "profiles")
    rounds = sorted((d for d in os.listdir(pdir) if d.startswith("r") and d[1:].isdigit()), reverse=True) \
        if os.path.isdir(pdir) else []
    for d in rounds:
        f = os.path.join(pdir, d, name)
        if os.path.exists(f):
            return f
    return None


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), or the platform's processor string."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def available_cpus():
    """CPUs this process may run on: its affinity mask, capped by a cgroup CPU quota
    (cgroup v2 cpu.max) -- on a GPU box os.cpu_count() shows the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    # the job's CPU share as the scheduler states it (the GPU pool sets OMP_NUM_THREADS to it)
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(L, M2, state, reps, budget_s=15.0, budget_1proc_s=8.0):
    """Oracle (NumPy restatement of the reference step, same diagnostics) on host cores.

    Bounded samples of the same workload (CPU timing plan 2):
      * 1 process stepping the workload's first replica for budget_1proc_s (value_1proc:
        the per-replica rate of the reference's own serial SPGG.run);
      * the reference's Pool parallelism (runner.py:142): min(available CPUs, replicas)
        processes, each stepping one replica of the workload for budget_s.
    The rates count the agent-steps completed inside the timed windows (after 3 warm-up
    iterations)."""
    import multiprocessing as mp
    avail = available_cpus()
    procs = max(1, min(avail, len(reps)))
    ctx = mp.get_context("spawn")   # spawned workers: the parent holds a HIP context; workers are NumPy only
    with ctx.Pool(1) as pool:
        one = pool.map(_cpu_job, [(L, M2, state, reps[0], budget_1proc_s)])[0]
    jobs = [(L, M2, state, reps[i % len(reps)], budget_s) for i in range(procs)]
    with ctx.Pool(procs) as pool:
        done = pool.map(_cpu_job, jobs)
    steps = sum(d[0] for d in done)
    wall = max(d[1] for d in done)
    agent_steps = steps * L * L
    out = {"value": agent_steps / wall, "unit": "agent-steps/s", "cores": procs, "kind": "port",
           "value_1proc": one[0] * L * L / one[1], "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
           "available_cpus": avail,
           "sample": f"oracle/spgg_oracle.py (NumPy, with diagnostics): {procs} processes (min of the "
                     f"{avail} CPUs available to this process and the workload's {len(reps)} replicas), each "
                     f"stepping one L={L} replica of the same workload for {budget_s:.0f} s after 3 warm-up "
                     f"iterations, {steps} iterations in {wall:.1f} s wall; value_1proc: one process alone, "
                     f"{one[0]} iterations in {one[1]:.1f} s"}
    # the oracle's speed relative to the reference's own SPGG.run on the same core
    # (tools/calibrate_cpu.py, survey container; the reference never travels)
    cal = os.path.join(ROOT, "profiles", "r03", "cpu_calibration.json")
    if os.path.exists(cal):
        c = json.load(open(cal))
        out["oracle_over_reference"] = c["oracle_over_reference"]
        out["reference_equivalent_value"] = out["value"] / c["oracle_over_reference"]
        out["reference_equivalent_value_1proc"] = out["value_1proc"] / c["oracle_over_reference"]
        out["calibration"] = (f"profiles/r03/cpu_calibration.json (measured in the survey container, where "
                              f"the reference can run; not this host): {c['workload']}; reference "
                              f"{c['reference_ms_per_iteration']:.1f} ms/iteration vs oracle "
                              f"{c['oracle_ms_per_iteration']:.1f}, one core of {c['cpu']}")
    return out


class _Budget(Exception):
    pass


def _cpu_job(job):
    """Step one replica with the oracle until the time budget is spent: (iterations, seconds)."""
    import numpy as np
    from oracle import spgg_oracle as O
    L, M2, state, p, budget = job
    op = O.Params(L=L, iterations=10 ** 9, use_second_order=M2, state_representation=state,
                  **{k: getattr(p, k) for k in ("r", "c", "cost", "alpha", "gamma", "epsilon",
                                                 "epsilon_decay", "epsilon_min", "influence_factor",
                                                 "lambda_epsilon", "delta_R_D", "R_min", "R_max",
                                                 "reward_weight_payoff", "rep_gain_C")})
    clock = {"t0": None, "n": 0}

    def on_step(i, *_):
        if i == 3:                       # warm-up done: start the timed window
            clock["t0"] = time.perf_counter()
        elif i > 3:
            clock["n"] += 1
            if time.perf_counter() - clock["t0"] >= budget:
                raise _Budget()

    try:
        O.run(op, np.random.RandomState(p.seed or 0), collect_snapshots=False, on_step=on_step)
    except _Budget:
        pass
    if clock["t0"] is None:              # absorbed during warm-up (not the bench workload)
        return 0, 1e-9
    return clock["n"], time.perf_counter() - clock["t0"]


FULL_RUN_ITERS = {"cfg2": 10000, "cfg3": 10000, "cfg4": 10000, "cfg5": 100000, "run100": 100001}


def full_run(L, M2, state, reps, rng, streams, T, offset, turn=256):
    """The configuration's whole run (BASELINE.json iterations) as a user runs it:
    BatchEngine.run() -- absorbing replicas, group retirement, host syncs every 256
    iterations (`turn`), the final flush -- timed from the first launch to the flush."""
    import numpy as np
    import torch
    from spgg_amd.engine import BatchEngine
    eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng=rng, streams=streams,
                      replica_offset=offset)
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run(chunk=turn, snapshots=False)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        stop = eng.stopped
        executed = np.where(stop == 0, eng.t - 1, stop - 1).astype(np.int64)
        absorbed = int(np.sum(stop != 0))
    finally:
        eng.close()
    agent_steps = float(executed.sum()) * L * L
    return {"iterations": T, "value": agent_steps / wall, "unit": "agent-steps/s", "seconds": wall,
            "executed_agent_steps": agent_steps, "replicas_absorbed": absorbed,
            "note": "whole run through BatchEngine.run (absorbing stops, group retirement, host syncs, flush)"}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the driver's own window (bench.py --steps 20 --warmup 5: iterations 6-25, eps 0.48 -> 0.40,
    # right after the engine is made); the line also carries the steady window 401-600 (eps at
    # eps_min from t = 390: what a 10,000-iteration run spends >96 % of its iterations in) and the
    # whole run
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-steady", action="store_true", help="skip the steady window (iterations 401-600)")
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rng", default="philox", choices=["philox", "mt19937"])
    ap.add_argument("--streams", type=int, default=None,
                    help="replica groups on concurrent HIP streams (default: auto)")
    ap.add_argument("--replicas", type=int, default=None,
                    help="experiment: first N replicas of the workload grid (cycled)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--full-run", type=int, default=-1,
                    help="also time the config's whole run (iterations; -1: BASELINE.json's, when it "
                         "takes under a minute at the measured step time; 0: off)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-mt", action="store_true",
                    help="skip the MT19937 (product-path) window reported beside a Philox line")
    args = ap.parse_args(argv)

    import numpy as np
    import torch
    import spgg_amd
    from spgg_amd import engine as E

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # the collectives' backend: RCCL ("nccl") on the GPUs; $SPGG_DIST_BACKEND=gloo for the tests of
    # this launch path (tests/test_bench_world_cpu.py on CPU; tests/test_gpu_launch_world2.py: two
    # ranks sharing one GPU, which RCCL refuses), whose collectives then run on host tensors
    backend = os.environ.get("SPGG_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()   # (counts devices without initialising one)
    if backend == "nccl" and local >= max(ndev, 1):
        raise SystemExit(f"LOCAL_RANK {local} but {ndev} GPU(s): one rank per GPU")
    torch.cuda.set_device(local % ndev if ndev else local)
    coll_dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    desc, L, M2, state, reps = workload(args.config, rank)
    if args.replicas:
        import dataclasses
        reps = [dataclasses.replace(reps[i % len(reps)], seed=(reps[i % len(reps)].seed or 0) + 7919 * (i // len(reps)))
                for i in range(args.replicas)]
        desc += f" [experiment: {args.replicas} replicas]"
    K, W = args.steps, args.warmup

    def window(rng, W=W, K=K):
        """W untimed + K timed iterations of a fresh engine in `rng` mode (barrier +
        synchronize on both sides; max over ranks): the executed agent-steps, times, layout."""
        eng = E.BatchEngine(L, K + W, reps, use_second_order=M2, state_representation=state, rng=rng,
                            streams=args.streams, replica_offset=rank * len(reps))
        mt_layout = None
        if rng == "mt19937":  # the draw generator's chains (spgg_mt_chains)
            mt_layout = {"chains_per_replica": eng.mt_layout[0], "iterations_per_chain": eng.mt_layout[1]}
        eng.step(W)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        # HIP events on the streams the step kernels run on (every replica group's), first start
        # to last end; the device is synchronised on both sides, so the groups' streams need no
        # ordering against the current stream (eng.step(ordered=False): two cross-stream waits
        # cost a 20-iteration window ~130 us, tools/window_timeline.py)
        streams = eng.launch_streams()
        ev0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
        ev1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
        t0 = time.perf_counter()
        for e, s_ in zip(ev0, streams):
            e.record(s_)
        eng.step(K, ordered=False)
        for e, s_ in zip(ev1, streams):
            e.record(s_)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        wall = time.perf_counter() - t0
        eng.check_status()   # a generator or persistent-barrier failure raises (no silent number)
        dev_ms = max(a_.elapsed_time(b_) for a_ in ev0 for b_ in ev1)
        stop = eng.stop_iter.cpu().numpy()
        # executed iterations in the timed window [W+1, W+K] per replica
        last = np.where(stop == 0, W + K, stop - 1)
        executed = np.clip(last - W, 0, K)
        agent_steps = float(executed.sum()) * L * L
        ncoop = eng.stats_folded()[:, :, 0].cpu().numpy()  # SPGG_ST_NCOOP per iteration slot
        coop = np.array([ncoop[k, int(last[k]) + 1] / (L * L) for k in range(len(reps))])
        # the window's cooperation-rate trace (iterations W+1 .. W+K; NaN after an absorbing stop)
        trace = ncoop[:, W + 1:W + K + 1] / (L * L)
        trace[np.arange(K)[None, :] + W + 1 > last[:, None] + 1] = np.nan
        tot = torch.tensor([agent_steps, wall], dtype=torch.float64, device=coll_dev)
        if dist:
            s_ = tot[:1].clone()
            dist.all_reduce(s_, op=dist.ReduceOp.SUM)
            w_ = tot[1:].clone()
            dist.all_reduce(w_, op=dist.ReduceOp.MAX)
            agent_steps_all, wall_max = float(s_.item()), float(w_.item())
        else:
            agent_steps_all, wall_max = agent_steps, wall
        out = dict(agent_steps=agent_steps, agent_steps_all=agent_steps_all, wall=wall, wall_max=wall_max,
                   dev_ms=dev_ms, coop=coop, trace=trace, mt_layout=mt_layout, resident=eng.resident,
                   groups=eng.G, waves=eng.waves, persistent=eng.persistent)
        eng.close()   # before the next engine, the full run and the CPU baseline's worker processes
        return out

    n_agents = len(reps) * L * L
    main_w = window(args.rng)
    agent_steps, wall, dev_ms = main_w["agent_steps"], main_w["wall"], main_w["dev_ms"]
    agent_steps_all, wall_max, mt_layout = main_w["agent_steps_all"], main_w["wall_max"], main_w["mt_layout"]
    # the path's only collective: every rank's per-replica final
    # cooperation rate and cooperation-rate trace, all-gathered (RCCL over xGMI on the GPUs)
    rows = np.concatenate([main_w["coop"][:, None], main_w["trace"]], axis=1)
    gathered_rows = rows[None]
    if dist:
        buf = torch.from_numpy(np.ascontiguousarray(rows)).to(coll_dev)
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
        gathered_rows = np.stack([p_.cpu().numpy() for p_ in parts])
    value = agent_steps_all / wall_max
    gathered_seed_max = max(int(p.seed or 0) for p in workload(args.config, world - 1)[4])
    per_step_dev_s = dev_ms / 1e3 / K
    step_agents = agent_steps / K
    achieved = ALGO_BYTES_PER_AGENT_STEP * step_agents / per_step_dev_s / 1e9
    achieved_wall = ALGO_BYTES_PER_AGENT_STEP * agent_steps / wall / 1e9
    resident, groups, waves = main_w["resident"], main_w["groups"], main_w["waves"]
    persistent = main_w["persistent"]
    # the step kernel the window ran: one launch per iteration and replica group, or (the whole
    # batch resident at once) one persistent launch per group for the K iterations
    step_kernel = (f"spgg_persist_kernel, {resident} concurrent launch(es) covering the {K} timed iterations "
                   f"(Q rows held in registers, a per-replica barrier between iterations)" if persistent else
                   f"spgg_step_kernel, {resident} concurrent launches per iteration (one per replica group/stream)")
    # the drop-in SPGG.run / sweep path: the device MT19937 stream, bit-identical to the reference
    mt_w = window("mt19937") if args.rng == "philox" and not args.no_mt else None
    steady = None
    if not args.no_steady and (W, K) != (400, 200):
        steady = window(args.rng, 400, 200)

    traffic = None
    # the traffic measured in this very window (profiles/r<NN>/traffic_<config>_w<a>-<b>.json), else
    # the config's generic file (a different window: named in traffic_unit)
    tfile = latest_profile(f"traffic_{args.config}_w{W + 1}-{W + K}.json") or latest_profile(
        f"traffic_{args.config}.json")
    if tfile and args.rng == "philox":
        # measured HBM bytes per agent-step (rocprofv3 PMC passes of this same command)
        traffic = json.load(open(tfile))["bytes_per_agent_step"] * step_agents
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "agent-steps/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": wall_max * 1e3 / K,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (reference init: S~Bernoulli(1/2), R=0, Q~U(-0.01,0.01))",
            "config": {"workload": desc, "window": f"iterations {W + 1}-{W + K}", "L": L, "replicas_per_gpu": len(reps),
                       "agents_per_gpu": n_agents, "second_order": M2, "state": state,
                       "rng": args.rng, "seeds_rank0": seed_range(reps), "seeds_all_ranks": f"0-{int(gathered_seed_max)}",
                       "streams_per_gpu": resident, "replica_groups": groups, "persistent": persistent,
                       "cache_waves": waves, "mt_chains": mt_layout,
                       "parallelism": f"replicas sharded over {world} GPU(s)"},
            "gather": {"replicas": int(gathered_rows.shape[0] * gathered_rows.shape[1]),
                       "bytes": int(gathered_rows.nbytes),
                       "mean_final_coop": float(np.mean(gathered_rows[:, :, 0])),
                       "what": "per-replica final cooperation rate + the window's cooperation-rate trace, "
                               "all_gather over every rank"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "time_base": "HIP events on every replica group's stream around the K timed iterations, first start to last end (device time per iteration)",
                         "achieved_wall": achieved_wall, "frac_wall": achieved_wall / HBM_PEAK_GBS,
                         "traffic_unit": "bytes per iteration (all replicas), from "
                                         + (os.path.relpath(tfile, ROOT) if tfile else "no PMC traffic file"),
                         "traffic_gbs": (traffic / per_step_dev_s / 1e9) if traffic else None,
                         "algorithmic_bytes_per_agent_step": ALGO_BYTES_PER_AGENT_STEP,
                         "kernel": (step_kernel if args.rng == "philox" else
                                    f"{step_kernel} + spgg_mt_gen_kernel (one launch per chunk of "
                                    f"{mt_layout['chains_per_replica']} chains x {mt_layout['iterations_per_chain']} "
                                    f"iterations per group) + spgg_mt_jump_kernel, on their own stream"),
                         "device_ms_per_step": per_step_dev_s * 1e3},
        }
        T_full = FULL_RUN_ITERS.get(args.config, 0) if args.full_run < 0 else args.full_run
        if args.full_run < 0 and wall_max / K * T_full > 60.0:
            T_full = 0
        if steady:
            sd = steady["dev_ms"] / 1e3 / 200
            line["steady_window"] = {
                "window": "iterations 401-600", "value": steady["agent_steps_all"] / steady["wall_max"],
                "unit": "agent-steps/s", "ms_per_step": steady["wall_max"] * 1e3 / 200,
                "device_ms_per_step": sd * 1e3,
                "roofline_frac": ALGO_BYTES_PER_AGENT_STEP * steady["agent_steps"] / 200 / sd / 1e9 / HBM_PEAK_GBS,
                "note": "the same workload after eps reached eps_min (t >= 390): the regime a 10,000-iteration "
                        "run spends >96 % of its iterations in; a fresh engine, 400 untimed iterations"}
        if mt_w:
            line["mt19937"] = {
                "value": mt_w["agent_steps_all"] / mt_w["wall_max"], "unit": "agent-steps/s",
                "ms_per_step": mt_w["wall_max"] * 1e3 / K, "mt_chains": mt_w["mt_layout"],
                "note": "the same K/W window with the device MT19937 stream (bit-identical to the reference's "
                        "numpy draws; what SPGG.run and the sweep use): spgg_step_kernel + the chained "
                        "draw generator (spgg_mt_gen_kernel, mt_jump_kernel) on its own stream"}
        if world == 1 and T_full > 0:
            line["full_run"] = full_run(L, M2, state, reps, args.rng, args.streams, T_full, 0)
            if mt_w:
                line["mt19937"]["full_run"] = full_run(L, M2, state, reps, "mt19937", args.streams, T_full, 0)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(L, M2, state, reps, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
