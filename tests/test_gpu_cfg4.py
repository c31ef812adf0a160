"""cfg4's own workload against the oracle (BASELINE.json configs[3]: L=200, second-order
neighbours, action state, the runner's constants, 8 replicas per GPU), and run_sharded's
mean_P against the reference's return value.

cfg4 runs with the planner's default layout (20 x 25 two-agent tiles, 2 replica groups) and
no environment overrides, on the device MT19937 stream: S, R, Q and the cooperation-rate /
switch / group-composition histories bit-exact, float histories within 1e-5 (north_star).
The action state (src/model/spgg.py:306-308) and the 12-offset NI (spgg.py:479-485) at this
size were otherwise only checked by Philox self-comparison."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from spgg_amd.engine import BatchEngine, ReplicaParams  # noqa: E402

FLOAT_TOL = dict(rtol=1e-5, atol=1e-9)
EXACT_KEYS = ("coop_rate_history", "switch_C_to_D", "switch_D_to_C", "epsilon_history_final") + tuple(
    f"group_comp_d{d}_history" for d in range(6))
FLOAT_KEYS = ("neighbor_influence_percent", "best_neighbor_second_order_percent", "avg_q_s0_c_history",
              "avg_q_s1_d_history", "cooperators_q_s0_c_history", "defectors_q_s1_d_history",
              "rep_avg_history_final", "avg_reward_C_history", "avg_reward_D_history", "it_records_final",
              "payoff_component_history", "rep_component_history")
OVERRIDES = ("SPGG_APT", "SPGG_STREAMS", "SPGG_CACHE_MB", "SPGG_CHUNK", "SPGG_ENQ_CHUNK", "SPGG_OWN_STREAMS",
             "SPGG_REP_F64", "SPGG_SKIP_DEAD")


def runner_params(**kw):
    base = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
                lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
                reward_weight_payoff=0.95, influence_factor=1.0, r=3.0)
    base.update(kw)
    return ReplicaParams(**base)


def _oracle_job(job):
    """One replica of the oracle (spawned worker: NumPy only)."""
    import numpy as np
    from oracle import spgg_oracle as O
    L, T, kw, seed, M2, state = job
    op = O.Params(L=L, iterations=T, use_second_order=M2, state_representation=state, **kw)
    rs = np.random.RandomState(seed)
    ds, fin = O.run(op, rs, collect_snapshots=False)
    return ds, {k: fin[k] for k in ("S", "R", "Q", "ret", "stop_iter")}


def _oracle_runs(L, T, reps, M2, state):
    import multiprocessing as mp
    keys = ("r", "c", "cost", "alpha", "gamma", "epsilon", "epsilon_decay", "epsilon_min", "influence_factor",
            "lambda_epsilon", "delta_R_D", "R_min", "R_max", "reward_weight_payoff", "rep_gain_C")
    jobs = [(L, T, {k: getattr(p, k) for k in keys}, p.seed, M2, state) for p in reps]
    with mp.get_context("spawn").Pool(min(len(jobs), 8)) as pool:   # (the box: 16 CPUs for the job)
        return pool.map(_oracle_job, jobs)


def test_cfg4_workload_bit_exact_vs_oracle(monkeypatch):
    for k in OVERRIDES:
        monkeypatch.delenv(k, raising=False)
    L, T = 200, 100
    reps = [runner_params(seed=s) for s in range(8)]   # BASELINE cfg4, rank 0's seeds
    eng = BatchEngine(L, T, reps, use_second_order=True, state_representation="action", rng="mt19937")
    try:
        assert eng.tile == (20, 25) and eng.G == 2, (eng.tile, eng.G)   # the planner's cfg4 layout
        assert eng.mt_layout[0] >= 1
        eng.run(snapshots=False)
        hist = eng.histories()
        finals = [eng.final_state(k) for k in range(len(reps))]
        keys = [eng.mt_state_host(k) for k in range(len(reps))]
    finally:
        eng.close()
    want = _oracle_runs(L, T, reps, True, "action")
    for k, (ds, fin) in enumerate(want):
        Q, R, S = finals[k]
        assert np.array_equal(S, fin["S"]), k
        assert np.array_equal(R, fin["R"]), k
        assert np.array_equal(Q, fin["Q"]), k
        h = hist[k]
        for key in EXACT_KEYS:
            assert np.array_equal(h[key], ds[key]), (k, key)
        for key in FLOAT_KEYS:
            np.testing.assert_allclose(h[key], ds[key], equal_nan=True, err_msg=f"{k} {key}", **FLOAT_TOL)
    # the continuing MT19937 key after the run = RandomState's after the same draws
    for k, p in enumerate(reps):
        rs = np.random.RandomState(p.seed)
        rs.uniform(-0.01, 0.01, (L, L, 2, 2))
        rs.randint(0, 2, (L, L))
        for _ in range(T):
            rs.rand(L, L)
            rs.randint(0, 2, (L, L))
        st = rs.get_state()
        assert np.array_equal(keys[k][0], np.asarray(st[1], dtype=np.uint32)) and keys[k][1] == st[2], k


def test_run_sharded_mean_P_matches_oracle():
    """run_sharded's summaries (distributed.replica_summaries): final rates, mean_P -- the mean
    payoff of the last iteration a replica started, SPGG.run's third return value
    (spgg.py:378,635-637) -- and the absorbing iteration, for a replica that runs to T and
    one that absorbs early (all-D at r=1), against the oracle's ret."""
    from spgg_amd import distributed as D
    L, T = 24, 700
    reps = [runner_params(r=3.0, seed=0), runner_params(r=1.0, seed=0)]
    summ, traces, eng = D.run_sharded(reps, L=L, iterations=T, use_second_order=False, rng="mt19937")
    eng.close()
    want = _oracle_runs(L, T, reps, False, "reputation")
    assert want[1][1]["stop_iter"] != 0 and want[0][1]["stop_iter"] == 0   # one absorbs, one does not
    for k, (ds, fin) in enumerate(want):
        c, d_, mp_ = fin["ret"]
        assert summ[k, 0] == c and summ[k, 1] == d_, k
        np.testing.assert_allclose(summ[k, 2], mp_, rtol=1e-12, atol=0)
        assert int(summ[k, 3]) == int(fin["stop_iter"]), k
        n = len(ds["coop_rate_history"])
        assert int(summ[k, 4]) == n
        np.testing.assert_array_equal(traces[k, :n], ds["coop_rate_history"])
        assert np.all(np.isnan(traces[k, n:]))
