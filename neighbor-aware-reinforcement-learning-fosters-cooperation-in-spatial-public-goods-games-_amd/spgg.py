"""Drop-in `SPGG` (src/model/spgg.py:39-637) whose run loop executes on the MI355X.

Same constructor signature, attributes, random-stream consumption, datasets
and return value as the reference, so `src/experiments/runner.py:88-105` can
construct and run it unchanged.  Construction stays on the host (it is the
reference's own one-off NumPy init: entropy reseed, Q ~ U(-0.01,0.01),
random population).  `run()` hands the continuing global MT19937 key to the
device, which reproduces every step of spgg.py:368-592 bit for bit in
libspgg_hip.so, then writes the reference's dataset layout.
"""
from __future__ import annotations

import os

import numpy as np

from . import algorithms as A
from .engine import BatchEngine, InitState, ReplicaParams, SNAPSHOT_ITERS
from .h5io import open_writer


def _sum5(A_):
    return A_ + np.roll(A_, -1, axis=0) + np.roll(A_, 1, axis=0) + np.roll(A_, -1, axis=1) + np.roll(A_, 1, axis=1)


def sum_position_and_neighbors(A_):
    """5-point periodic sum (spgg.py:23-36); host utility kept for API parity."""
    return _sum5(A_)


class SPGG:
    """Spatial Public Goods Game with RL, reputation and neighbor influence."""

    save_png = True  # strategy PNGs at snapshot iterations (spgg.py:552-559)

    def __init__(self, r=2, c=1, cost=0.5, K=0.1, L=50, iterations=1000,
                 num_of_strategies=2, population_type=0, S_in_one=None,
                 alpha=0.1, gamma=0.9, epsilon=0.5, epsilon_decay=0.995,
                 epsilon_min=0.01, influence_factor=1.0, use_second_order=True,
                 lambda_epsilon=0.01, delta_R_C=1, delta_R_D=1, R_min=-10,
                 R_max=10, reward_weight_payoff=1.0, rep_gain_C=0.5,
                 state_representation='reputation', algorithm='qlearning', **params):
        np.random.seed()  # spgg.py:98: entropy reseed of the global MT19937

        all_params = dict(locals(), **params)
        del all_params['self'], all_params['params']
        self.params = all_params
        for key in self.params:
            setattr(self, key, self.params[key])
        self.reward_weight_rep = 1 - self.reward_weight_payoff

        if isinstance(algorithm, str):
            self.algorithm = A.create_algorithm(algorithm, alpha, gamma, epsilon,
                                                epsilon_decay, epsilon_min, **params)
        elif A.is_operator(algorithm):
            # the plug-in point (spgg.py:115-116): one of the operators the device step
            # implements, this package's or the reference's own; a custom operator raises
            # ValueError here instead of running the built-in math (algorithms.operator_kind)
            A.operator_kind(algorithm)
            self.algorithm = algorithm
        else:
            raise ValueError(f"algorithm must be str or RLAlgorithm, got {type(algorithm)}")

        self.q_table = np.random.uniform(low=-0.01, high=0.01, size=(L, L, 2, 2))
        if hasattr(self.algorithm, 'initialize_q_tables'):
            self.algorithm.initialize_q_tables(self.q_table.shape)
            self.q_table = self.algorithm.get_combined_q_table()
        self.R = np.zeros((L, L))
        self.cache = {}
        self._Sn = S_in_one
        self.create_population()

        self.track_positions = track_positions(L)
        self.q_history = {pos: {'q_c': [], 'q_d': []} for pos in self.track_positions}
        self.it_records = []
        self.epsilon_history = []
        self.rep_avg_history = []
        self.influence_counts = []
        self.best_neighbor_type_history = []
        self.normlize_max = 4 * r
        self.normlize_min = r - 5
        max_pow = int(np.floor(np.log10(self.iterations)))  # noqa: F841 (spgg.py:152)
        self.snapshot_iters = set(SNAPSHOT_ITERS)
        self.folder = None

    def create_population(self):
        """spgg.py:158-164."""
        L = self.L
        if self._Sn is None:
            self._Sn = np.random.randint(0, 2, size=(L, L))
        self._S = [(self._Sn == j).astype(int) for j in range(self.num_of_strategies)]
        return self._S

    def generate_cache_key(self, *args):
        return hash(args)

    # -- run -----------------------------------------------------------------
    def _replica_params(self):
        alg = self.algorithm
        return ReplicaParams(
            r=self.r, c=self.c, cost=self.cost, alpha=self.alpha, gamma=self.gamma,
            epsilon=alg.epsilon, epsilon_decay=alg.epsilon_decay, epsilon_min=alg.epsilon_min,
            influence_factor=self.influence_factor, lambda_epsilon=self.lambda_epsilon,
            delta_R_D=self.delta_R_D, R_min=self.R_min, R_max=self.R_max,
            reward_weight_payoff=self.reward_weight_payoff, rep_gain_C=self.rep_gain_C,
            alg_alpha=alg.alpha, alg_gamma=alg.gamma)

    def run(self, filename):
        """Run the simulation on the GPU and write the datasets (spgg.py:325-637).

        Returns (final_coop_rate, final_def_rate, mean_payoff) as numpy float64.
        """
        kind = A.canonical_name(self.algorithm)
        L = self.L
        S0 = np.asarray(self._Sn)
        n0 = int(np.sum(S0 == 0))
        absorbing0 = n0 == 0 or n0 == L * L
        state_rep = self.state_representation
        if state_rep not in ('reputation', 'action'):
            if not absorbing0:  # the reference raises at the first get_state (spgg.py:309)
                raise ValueError(f"Unknown state_representation: {state_rep}. "
                                 f"Must be 'reputation' or 'action'")
            state_rep = 'reputation'
        g = np.random.get_state()
        tables = None
        if kind == "double_qlearning":
            tables = (np.asarray(self.algorithm.q_table_1, dtype=np.float64),
                      np.asarray(self.algorithm.q_table_2, dtype=np.float64))
        init = InitState(Q=np.asarray(self.q_table, dtype=np.float64), S=S0, tables=tables,
                         mt_key=np.asarray(g[1], dtype=np.uint32), mt_pos=int(g[2]))
        iters = int(self.iterations)
        eng = BatchEngine(L, max(iters, 1), [self._replica_params()],
                          use_second_order=bool(self.use_second_order),
                          state_representation=state_rep, rng="mt19937", init=[init],
                          algorithm=kind)
        if iters < 1:
            eng.T = 0
        snapshots_dir = os.path.join(self.folder, 'plots', 'snapshots') if self.folder else 'snapshots'
        os.makedirs(snapshots_dir, exist_ok=True)
        try:
            eng.run(snapshots=True, png=self.save_png)
            hist = eng.histories()[0]
            Q, R, S = eng.final_state(0)
            tables = eng.final_tables(0) if kind == "double_qlearning" else None
            last = eng.last_iteration(0)
            P = eng.payoff_at(last)[0] if last >= 1 else None
            key, pos = eng.mt_state_host(0)
            m = len(hist["epsilon_history_final"])
            eps_after = float(eng.eps_host[0, m + 1]) if m > 0 else None
            snaps, frames = eng.snapshots[0], eng.png_frames[0]
        finally:
            eng.close()

        if self.save_png and frames:
            _write_pngs(frames, snapshots_dir)

        # state after the run, as the reference leaves it
        self.q_table, self.R, self._Sn = Q, R, S
        if tables is not None:  # the operator's own tables (spgg.py:496-502)
            self.algorithm.q_table_1, self.algorithm.q_table_2 = tables
        self._S = [(S == j).astype(int) for j in range(self.num_of_strategies)]
        self.cache = {}
        if P is not None:
            self.P = P
        if eps_after is not None:
            self.algorithm.epsilon = eps_after
            self.epsilon = eps_after
        np.random.set_state((g[0], key, pos, g[3], g[4]))

        # the datasets last: the reference fills its file after the loop, so a write
        # error (duplicate tracked positions at L <= 2) leaves the state above in place
        write_datasets(filename, hist, snaps, S, R, self.R_min, self.R_max, self.track_positions)

        S_coop = (S == 0).astype(int)
        S_def = (S == 1).astype(int)
        return (np.sum(S_coop) / (L * L), np.sum(S_def) / (L * L), np.mean(P))



HISTORY_DATASETS = ("it_records_final", "epsilon_history_final", "rep_avg_history_final",
                    "coop_rate_history", "switch_C_to_D", "switch_D_to_C",
                    "neighbor_influence_percent", "payoff_component_history",
                    "rep_component_history", "best_neighbor_second_order_percent",
                    "reputation_reward_ratio", "avg_reward_C_history", "avg_reward_D_history")


def write_datasets(filename, hist, snaps, S, R, R_min, R_max, track_positions):
    """The dataset layout `SPGG.run` writes (spgg.py:594-633): snapshots, the
    per-iteration histories, the never-filled tracked-position Q datasets and
    the final state.  Shared by SPGG.run and the batched sweep runner."""
    with open_writer(filename) as data_file:
        for i in sorted(snaps):
            Ri, Si = snaps[i]
            data_file.create_dataset(f"R_snapshot_{i}", data=Ri)
            h, bins = np.histogram(Ri, bins=20, range=(R_min, R_max))
            data_file.create_dataset(f"rep_hist_{i}", data=h)
            data_file.create_dataset(f"rep_bins_{i}", data=bins)
            data_file.create_dataset(f"Sn_snapshot_{i}", data=Si)
        for name in HISTORY_DATASETS:
            data_file.create_dataset(name, data=hist[name])
        for d in range(6):
            data_file.create_dataset(f"group_comp_d{d}_history", data=hist[f"group_comp_d{d}_history"])
        for grp in ("cooperators", "defectors"):
            for s in ("s0", "s1"):
                for a in ("c", "d"):
                    k = f"{grp}_q_{s}_{a}_history"
                    data_file.create_dataset(k, data=hist[k])
        for s in ("s0", "s1"):
            for a in ("c", "d"):
                k = f"avg_q_{s}_{a}_history"
                data_file.create_dataset(k, data=hist[k])
        for p_ in track_positions:  # never filled by the reference (spgg.py:345,620-622)
            data_file.create_dataset(f"q_c_pos_{p_[0]}_{p_[1]}_final", data=np.array([]))
            data_file.create_dataset(f"q_d_pos_{p_[0]}_{p_[1]}_final", data=np.array([]))
        data_file.create_dataset("Sn_final", data=S)
        data_file.create_dataset("R_final", data=R)
        h, bins = np.histogram(R, bins=20, range=(R_min, R_max))
        data_file.create_dataset("rep_hist_final", data=h)
        data_file.create_dataset("rep_bins_final", data=bins)
        data_file.create_dataset("cluster_sizes", data=cluster_sizes(S))


def track_positions(L):
    """Positions whose Q the reference meant to track (spgg.py:143)."""
    return [(L // 2, L // 2), (L // 4, L // 4), (3 * L // 4, 3 * L // 4)]


def cluster_sizes(S):
    """Sizes of 4-connected non-periodic cooperator clusters, label order (spgg.py:631-633).

    One bincount instead of the reference's O(k*L^2) per-label comprehension.
    """
    from scipy.ndimage import label
    lab, n = label(S == 0)
    return np.bincount(lab.ravel(), minlength=n + 1)[1:].astype(np.int64)


def _write_pngs(frames, snapshots_dir):
    """Strategy snapshot images (spgg.py:14-20, 552-559)."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib as mpl
        import matplotlib.pyplot as plt
    except Exception:  # noqa: BLE001 - matplotlib is optional for the hot path
        return
    cmap = mpl.colors.ListedColormap(["#eeeeee", "#111111"], N=2)
    for i, Sn in sorted(frames.items()):
        fig, ax = plt.subplots(figsize=(5, 5))
        ax.imshow(Sn, cmap=cmap, interpolation='nearest')
        ax.set_title(f"Strategy at iter={i}")
        ax.axis('off')
        fig.savefig(os.path.join(snapshots_dir, f"snapshot_{i}.png"))
        plt.close(fig)
