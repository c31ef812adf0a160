"""Batched experiment sweeps: the caller of the hot path, MI355X-native.

Restates the reference's experiment layer -- `src/experiments/runner.py:11-156`
(folder naming, `run_one_experiment`, `run_experiments`), `src/config_loader.py:
11-211` (`load_config`, `generate_param_combinations`, `get_model_params`) and
the `scripts/run_experiments.py:16-97` entry point -- with one change of
execution model.  The reference runs every parameter tuple as its own SPGG in
a `multiprocessing.Pool` worker (one L=100 lattice per CPU core).  Here tuples
that share a step-kernel configuration (second-order flag, state
representation, RL operator) become the replicas of ONE `BatchEngine`, so a
single launch per iteration steps all of them, and the batches are sharded
over the node's GPUs (one process per GPU; under torchrun, one rank per GPU
with an RCCL all-gather of the per-experiment summaries at the end).

Every experiment still gets its own folder, named exactly as the reference
names it, holding the files `SPGG.run` writes (data/experiment_data.h5 with the
reference's datasets, plots/snapshots/*.png); the return value keeps the
reference's `(params, (final_coop_ratio, final_rep_mean))` shape.
"""
from __future__ import annotations

import copy
import os
import sys
from itertools import product
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

ALGORITHMS = ("qlearning", "sarsa", "expected_sarsa", "double_qlearning")
EXPERIMENT_TYPES = ("figure_2_3_4", "figure_6_7_8_9", "all_figures", "custom")

# Constants run_one_experiment passes to SPGG besides the swept values (runner.py:88-101).
RUNNER_MODEL = dict(c=1, cost=1, iterations=100001, L=100, num_of_strategies=2, K=0.1,
                    population_type=0, gamma=0.9, epsilon=0.5, epsilon_decay=0.99,
                    epsilon_min=0.01, lambda_epsilon=0.01, delta_R_C=1, delta_R_D=1,
                    R_min=-10, R_max=10)

# The values of the reference's config/default_config.yaml, used when no file is given.
DEFAULT_CONFIG: Dict[str, Any] = {
    "model": {"r": 3.0, "c": 1.0, "cost": 1.0, "L": 100, "iterations": 100001,
              "num_of_strategies": 2, "K": 0.1, "population_type": 0},
    "rl": {"algorithm": "qlearning", "alpha": 0.8, "gamma": 0.9, "epsilon": 0.5,
           "epsilon_decay": 0.99, "epsilon_min": 0.01, "state_representation": "reputation"},
    "neighbor_influence": {"influence_factor": 1.0, "use_second_order": True, "lambda_epsilon": 0.01},
    "reputation": {"delta_R_C": 1.0, "delta_R_D": 1.0, "R_min": -10, "R_max": 10, "rep_gain_C": 1.0},
    "reward": {"reward_weight_payoff": 0.95},
    "experiments": {
        "figure_2_3_4": {"r": 3.6, "kappas": [0.0, 0.5, 1.0, 1.5, 2.0],
                         "use_second_order": [False, True], "reward_weight_payoff": 1.0},
        "figure_6_7_8_9": {"r": 3.0, "use_second_order": [False, True]},
        "all_figures": None,
        "custom": {"r_values": [1.0, 2.0, 3.0, 4.0, 5.0], "kappa_values": [0.0, 0.5, 1.0, 1.5, 2.0],
                   "use_second_order": [False, True], "reward_weight_payoff_values": [0.83, 0.95, 1.0]},
    },
    "output": {"base_dir": "results", "save_snapshots": True,
               "snapshot_iterations": [1, 10, 100, 1000, 5000, 10000, 20000, 30000, 40000],
               "save_plots": True},
}


# ---------------------------------------------------------------------------
# configuration (config_loader.py)

def load_config(config_path: Optional[str] = None) -> Dict[str, Any]:
    """YAML config (safe loader), or the reference's defaults when no path is given
    (config_loader.py:11-36).  A missing file raises FileNotFoundError."""
    if config_path is None:
        return copy.deepcopy(DEFAULT_CONFIG)
    if not os.path.exists(config_path):
        raise FileNotFoundError(f"Config file not found: {config_path}")
    import yaml
    with open(config_path) as f:
        return yaml.safe_load(f)


def _as_list(x):
    return [x] if isinstance(x, str) else list(x)


def generate_param_combinations(config: Dict[str, Any], experiment_type: str = "custom") -> List[Tuple]:
    """Sorted, de-duplicated 7-tuples (r, kappa, use_second_order, alpha, w_P,
    rep_gain_C, state_representation) of an experiment type (config_loader.py:39-156)."""
    rl = config.get("rl", {})
    exps = config.get("experiments", {}) or {}
    alpha = rl.get("alpha", 0.8)
    gain = config.get("reputation", {}).get("rep_gain_C", 1.0)
    state0 = rl.get("state_representation", "reputation")

    def fig234():
        f = exps.get("figure_2_3_4", {}) or {}
        states = _as_list(f.get("state_representation", [state0]))
        return [(f.get("r", 3.6), k, so, alpha, f.get("reward_weight_payoff", 1.0), gain, st)
                for k, so, st in product(f.get("kappas", [0.0, 0.5, 1.0, 1.5, 2.0]),
                                         f.get("use_second_order", [False, True]), states)]

    def fig6789():
        f = exps.get("figure_6_7_8_9", {}) or {}
        r = f.get("r", 3.0)
        orders = f.get("use_second_order", [False, True])
        states = _as_list(f.get("state_representation", [state0]))
        out = []
        # sole reputation (kappa 0, w_P 0.95), sole NI (kappa 1, w_P 1.0), hybrid (kappa 1, w_P 0.95)
        for kappa, w_p in ((0.0, 0.95), (1.0, 1.0), (1.0, 0.95)):
            out += [(r, kappa, so, alpha, w_p, gain, st) for so, st in product(orders, states)]
        return out

    if experiment_type == "figure_2_3_4":
        combos = fig234()
    elif experiment_type == "figure_6_7_8_9":
        combos = fig6789()
    elif experiment_type == "all_figures":
        combos = fig234() + fig6789()
    elif experiment_type == "custom":
        f = exps.get("custom", {}) or {}
        states = _as_list(f.get("state_representation", [state0]))
        combos = [(r, k, so, alpha, w_p, gain, st) for r, k, so, w_p, st in product(
            f.get("r_values", [1.0, 2.0, 3.0, 4.0, 5.0]), f.get("kappa_values", [0.0, 0.5, 1.0, 1.5, 2.0]),
            f.get("use_second_order", [False, True]), f.get("reward_weight_payoff_values", [0.83, 0.95, 1.0]),
            states)]
    else:
        raise ValueError(f"Unknown experiment type: {experiment_type}")
    return sorted(set(combos))


def get_model_params(config: Dict[str, Any], **overrides) -> Dict[str, Any]:
    """SPGG keyword arguments from a config, with overrides (config_loader.py:159-211)."""
    sec = {k: config.get(k, {}) or {} for k in ("model", "rl", "neighbor_influence", "reputation", "reward")}
    spec = (("model", "r", 2.0), ("model", "c", 1.0), ("model", "cost", 0.5), ("model", "K", 0.1),
            ("model", "L", 50), ("model", "iterations", 1000), ("model", "num_of_strategies", 2),
            ("model", "population_type", 0), ("rl", "algorithm", "qlearning"), ("rl", "alpha", 0.1),
            ("rl", "gamma", 0.9), ("rl", "epsilon", 0.5), ("rl", "epsilon_decay", 0.995),
            ("rl", "epsilon_min", 0.01), ("rl", "state_representation", "reputation"),
            ("neighbor_influence", "influence_factor", 1.0), ("neighbor_influence", "use_second_order", True),
            ("neighbor_influence", "lambda_epsilon", 0.01), ("reputation", "delta_R_C", 1.0),
            ("reputation", "delta_R_D", 1.0), ("reputation", "R_min", -10), ("reputation", "R_max", 10),
            ("reward", "reward_weight_payoff", 1.0), ("reputation", "rep_gain_C", 0.5))
    params = {key: sec[s].get(key, default) for s, key, default in spec}
    params.update(overrides)
    return params


# ---------------------------------------------------------------------------
# experiments (runner.py)

def get_folder_name(r: float, kappa: float, use_second_order: bool, alpha: float,
                    reward_weight_payoff: float, rep_gain_C: float,
                    state_representation: str = "reputation", algorithm: str = "qlearning") -> str:
    """Result folder of one experiment, character for character as runner.py:11-45."""
    state = "_action" if state_representation == "action" else ""
    algo = "" if algorithm == "qlearning" else f"_{algorithm}"
    return (f"results_r{r}_inf{kappa}_order{use_second_order}_alpha{alpha}_"
            f"rw{reward_weight_payoff:.2f}_rgC{rep_gain_C:.2f}{state}{algo}")


def unpack(params: Tuple) -> Tuple:
    """8-tuple (r, kappa, M2, alpha, w_P, gain, state, algorithm) from the 6/7/8-tuple
    forms run_one_experiment accepts (runner.py:62-72)."""
    if len(params) == 8:
        return tuple(params)
    if len(params) == 7:
        return tuple(params) + ("qlearning",)
    if len(params) == 6:
        return tuple(params) + ("reputation", "qlearning")
    raise ValueError(f"Unexpected parameter format: {params}")


def make_folders(folder: str):
    """runner.py:79-86: the experiment's directory tree (created once)."""
    if not os.path.exists(folder):
        for sub in ("", "configurations", "reputations", "plots", os.path.join("plots", "snapshots"), "data"):
            os.makedirs(os.path.join(folder, sub), exist_ok=True)


def _done_line(p8):
    r, kappa, so, alpha, w_p, gain, state, algorithm = p8
    label = "action" if state == "action" else "rep"
    return (f"Done: r={r}, κ={kappa}, M={2 if so else 1}, α={alpha}, w_P={w_p}, ΔR_C={gain}, "
            f"state={label}, algo={algorithm}")


def run_one_experiment(params: Tuple, **model_overrides) -> Tuple[Tuple, Tuple[float, float]]:
    """One experiment through the drop-in SPGG (runner.py:48-111): same folder, files,
    print and return value.  model_overrides replace RUNNER_MODEL entries (e.g. L)."""
    from .spgg import SPGG
    p8 = unpack(params)
    r, kappa, so, alpha, w_p, gain, state, algorithm = p8
    folder = get_folder_name(*p8)
    make_folders(folder)
    kw = dict(RUNNER_MODEL, **model_overrides)
    spgg = SPGG(r=r, alpha=alpha, influence_factor=kappa, use_second_order=so,
                reward_weight_payoff=w_p, rep_gain_C=gain, state_representation=state,
                algorithm=algorithm, **kw)
    spgg.folder = folder
    coop, _def, _p = spgg.run(os.path.join(folder, "data", "experiment_data.h5"))
    rep_mean = spgg.rep_avg_history[-1] if spgg.rep_avg_history else 0
    print(_done_line(p8))
    return params, (coop, rep_mean)


def _replica(p8, kw, seed):
    from .engine import ReplicaParams
    r, kappa, _so, alpha, w_p, gain, _state, _alg = p8
    return ReplicaParams(r=r, c=kw["c"], cost=kw["cost"], alpha=alpha, gamma=kw["gamma"],
                         epsilon=kw["epsilon"], epsilon_decay=kw["epsilon_decay"],
                         epsilon_min=kw["epsilon_min"], influence_factor=kappa,
                         lambda_epsilon=kw["lambda_epsilon"], delta_R_D=kw["delta_R_D"],
                         R_min=kw["R_min"], R_max=kw["R_max"], reward_weight_payoff=w_p,
                         rep_gain_C=gain, seed=seed)


def run_batch(param_list: Sequence[Tuple], seeds: Optional[Sequence[Optional[int]]] = None,
              device=None, save_png: bool = True, verbose: bool = True, progress=None,
              **model_overrides) -> List[Tuple[Tuple, Tuple[float, float]]]:
    """Run experiments on ONE GPU as replica batches; results in input order.

    Tuples sharing (use_second_order, state_representation, algorithm) run as
    the replicas of one BatchEngine (device MT19937: each replica's draws are
    exactly those its own `SPGG(...).run()` would make).  seeds[i] seeds
    experiment i's RandomState; None = entropy, as the reference's
    `np.random.seed()` (spgg.py:98)."""
    import torch
    from .engine import BatchEngine, reference_init
    from .spgg import _write_pngs, track_positions, write_datasets
    from .algorithms import canonical_name
    kw = dict(RUNNER_MODEL, **model_overrides)
    L, iters = int(kw["L"]), int(kw["iterations"])
    p8s = [unpack(p) for p in param_list]
    seeds = list(seeds) if seeds is not None else [None] * len(p8s)
    if len(seeds) != len(p8s):
        raise ValueError("one seed (or None) per parameter tuple")
    for p in p8s:
        if p[6] not in ("reputation", "action"):
            raise ValueError(f"Unknown state_representation: {p[6]}. Must be 'reputation' or 'action'")
        if canonical_name(p[7]) not in ALGORITHMS:
            raise ValueError(f"Unknown algorithm: {p[7]}")
    if device is not None:
        torch.cuda.set_device(device)
    groups: Dict[Tuple, List[int]] = {}
    for i, p in enumerate(p8s):
        groups.setdefault((bool(p[2]), p[6], canonical_name(p[7])), []).append(i)
    out: List[Optional[Tuple]] = [None] * len(p8s)
    for (so, state, alg), idx in groups.items():
        reps = [_replica(p8s[i], kw, seeds[i]) for i in idx]
        inits = [reference_init(L, np.random.RandomState(seeds[i]), algorithm=alg) for i in idx]
        eng = BatchEngine(L, max(iters, 1), reps, use_second_order=so, state_representation=state,
                          rng="mt19937", init=inits, algorithm=alg)
        try:
            eng.run(snapshots=True, png=save_png, progress=progress)
            hist = eng.histories()
            for k, i in enumerate(idx):
                folder = get_folder_name(*p8s[i])
                make_folders(folder)
                _q, R, S = eng.final_state(k)
                write_datasets(os.path.join(folder, "data", "experiment_data.h5"), hist[k], eng.snapshots[k],
                               S, R, kw["R_min"], kw["R_max"], track_positions(L))
                if save_png and eng.png_frames[k]:
                    _write_pngs(eng.png_frames[k], os.path.join(folder, "plots", "snapshots"))
                coop = float(np.sum(S == 0)) / (L * L)
                out[i] = (param_list[i], (coop, 0))  # SPGG.rep_avg_history is never filled (spgg.py:140)
                if verbose:
                    print(_done_line(p8s[i]))
        finally:
            eng.close()
    return out


def _gpu_worker(args):
    root, device, params, seeds, save_png, overrides = args
    if root not in sys.path:
        sys.path.insert(0, root)
    import spgg_amd  # noqa: F401  (package import shim at the repository root)
    from spgg_amd.sweep import run_batch
    return run_batch(params, seeds=seeds, device=device, save_png=save_png, verbose=True, **overrides)


def run_experiments(param_combinations: List[Tuple], num_processes: Optional[int] = None,
                    use_progress_bar: bool = True, seeds: Optional[Sequence[Optional[int]]] = None,
                    devices: Optional[Sequence[int]] = None, save_png: bool = True,
                    **model_overrides) -> List[Tuple]:
    """runner.py:114-156 with GPU batches instead of a CPU process pool.

    Sharding (contiguous blocks of the tuple list, distributed.shard_range):
      * under torch.distributed (torchrun, one rank per GPU): this rank's block on
        its GPU, then an all-gather of (final_coop, final_rep_mean) -- every rank
        returns the full list;
      * otherwise over `devices` (default: every visible GPU, at most
        num_processes of them), one spawned process per GPU;
      * one GPU: in this process.
    Results are in input order (the reference's Pool.map order)."""
    import torch
    from .distributed import gather_rows, shard_range
    params = list(param_combinations)
    seeds = list(seeds) if seeds is not None else [None] * len(params)
    bar = None
    if use_progress_bar:
        try:
            from tqdm import tqdm
            bar = tqdm(total=int(dict(RUNNER_MODEL, **model_overrides)["iterations"]), desc="Running simulations")
        except ImportError:
            print("tqdm not available, running without progress bar")

    def progress(t):
        if bar is not None:
            bar.n = t
            bar.refresh()

    import torch.distributed as dist
    from .distributed import local_device
    try:
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            world, rank = dist.get_world_size(), dist.get_rank()
            a, b = shard_range(len(params), world, rank)
            # this rank's GPU (LOCAL_RANK), before its engine exists; only its own block runs here
            local = run_batch(params[a:b], seeds[a:b], device=local_device(), save_png=save_png,
                              progress=progress, **model_overrides)
            rows = np.array([[res[0], res[1]] for _, res in local], dtype=np.float64).reshape(-1, 2)
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
            allr = gather_rows(rows, len(params), device=dev)
            return [(params[i], (float(allr[i, 0]), allr[i, 1])) for i in range(len(params))]
        if devices is None:
            n_dev = torch.cuda.device_count()
            devices = list(range(max(1, min(n_dev, num_processes or n_dev))))
        devices = list(devices)
        if len(devices) <= 1 or len(params) <= 1:
            return run_batch(params, seeds, device=devices[0] if devices else None, save_png=save_png,
                             progress=progress, **model_overrides)
        import multiprocessing as mp
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        jobs = []
        for w, d in enumerate(devices):
            a, b = shard_range(len(params), len(devices), w)
            if b > a:
                jobs.append((root, d, params[a:b], seeds[a:b], save_png, dict(model_overrides)))
        with mp.get_context("spawn").Pool(len(jobs)) as pool:
            parts = pool.map(_gpu_worker, jobs)
        return [x for part in parts for x in part]
    finally:
        if bar is not None:
            bar.close()


# ---------------------------------------------------------------------------
# entry point (scripts/run_experiments.py)

def resolve_algorithms(requested: Optional[Sequence[str]], config: Dict[str, Any]) -> List[str]:
    """Algorithms to run: --algorithms (names or 'all') or the config's (run_experiments.py:46-63)."""
    if requested:
        req = [a.lower() for a in requested]
        if "all" in req:
            algs = list(ALGORITHMS)
        else:
            bad = [a for a in req if a not in ALGORITHMS]
            if bad:
                raise ValueError(f"Unknown algorithms requested: {bad}. Choose from {list(ALGORITHMS)} or 'all'.")
            algs = req
    else:
        algs = [config.get("rl", {}).get("algorithm", "qlearning").lower()]
    return sorted(set(algs), key=ALGORITHMS.index)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Run SPGG experiments (batched on MI355X)")
    ap.add_argument("--config", type=str, default=None)
    ap.add_argument("--experiment-type", choices=EXPERIMENT_TYPES, default="custom")
    ap.add_argument("--num-processes", type=int, default=None, help="GPUs to use (default: all visible)")
    ap.add_argument("--no-progress", action="store_true")
    ap.add_argument("--algorithms", type=str, nargs="+", default=None)
    args = ap.parse_args(argv)
    config = load_config(args.config)
    algs = resolve_algorithms(args.algorithms, config)
    combos = [(*p, a) for p in generate_param_combinations(config, args.experiment_type) for a in algs]
    # under torchrun (WORLD_SIZE > 1): one rank per GPU, each running its block of the
    # tuples (run_experiments' distributed branch), instead of every rank fanning out
    # over all GPUs
    from .distributed import init_from_env
    import torch.distributed as dist
    owned = init_from_env()
    lead = not dist.is_initialized() or dist.get_rank() == 0
    try:
        if lead:
            print(f"Algorithms selected: {', '.join(algs)}")
            print(f"Total parameter combinations: {len(combos)}")
        results = run_experiments(combos, num_processes=args.num_processes,
                                  use_progress_bar=lead and not args.no_progress)
        if lead:
            print(f"\nCompleted {len(results)} experiments")
    finally:
        if owned:
            dist.destroy_process_group()
    return results


if __name__ == "__main__":
    main()
