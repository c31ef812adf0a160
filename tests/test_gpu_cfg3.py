"""The headline batch itself under parity: BASELINE.json configs[2] / bench.py's default
workload (105 x L=200 replicas: r in {2.0..5.0} x kappa in {0, 0.5, 1} x 5 seeds, M=1,
reputation state, w_P=1.0), run exactly as the bench plans it -- two auto-planned replica
groups on concurrent streams, 40 x 25 tiles through the compile-time-width (TWC=40) step
kernel, the kappa == 0 replicas without pending NI records -- in the reference's own random
stream (device MT19937), against the oracle (reference spgg.py:368-592)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import bench  # noqa: E402  (repository root)
import spgg_amd  # noqa: E402
from spgg_amd.engine import BatchEngine  # noqa: E402
from oracle import spgg_oracle as O  # noqa: E402

FLOAT_TOL = dict(rtol=1e-5, atol=1e-9)
T = 20
EXACT = ("coop_rate_history", "switch_C_to_D", "switch_D_to_C", "epsilon_history_final") + tuple(
    f"group_comp_d{d}_history" for d in range(6))
APPROX = ("neighbor_influence_percent", "rep_avg_history_final", "it_records_final", "avg_reward_C_history",
          "avg_reward_D_history", "payoff_component_history", "avg_q_s0_c_history", "avg_q_s1_d_history",
          "cooperators_q_s0_d_history", "defectors_q_s1_c_history")


def _oracle(p, L, M2, state):
    op = O.Params(L=L, iterations=T, use_second_order=M2, state_representation=state,
                  **{k: getattr(p, k) for k in ("r", "c", "cost", "alpha", "gamma", "epsilon",
                                                 "epsilon_decay", "epsilon_min", "influence_factor",
                                                 "lambda_epsilon", "delta_R_D", "R_min", "R_max",
                                                 "reward_weight_payoff", "rep_gain_C")})
    return O.run(op, np.random.RandomState(p.seed), collect_snapshots=False)


def test_cfg3_batch_mt19937_vs_oracle():
    _, L, M2, state, reps = bench.workload("cfg3", 0)
    assert len(reps) == 105 and L == 200
    eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng="mt19937")
    try:
        assert eng.G == 2 and eng.waves == 1, (eng.G, eng.waves)      # the bench's plan
        assert eng.tile == (40, 25)                                     # TWC=40 kernel instance
        assert sum(p.influence_factor == 0.0 for p in reps) == 35
        eng.run(snapshots=False)
        hs = eng.histories()
        # one replica per (r, kappa) cell, seeds rotated so every seed and both groups appear
        cells = [i * 15 + j * 5 + (i + j) % 5 for i in range(7) for j in range(3)]
        for k in cells:
            p = reps[k]
            ds, fin = _oracle(p, L, M2, state)
            Q, R, S = eng.final_state(k)
            assert np.array_equal(S, fin["S"]), k
            assert np.array_equal(R, fin["R"]), k
            assert np.array_equal(Q, fin["Q"]), k
            for key in EXACT:
                assert np.array_equal(hs[k][key], ds[key]), (k, key)
            for key in APPROX:
                np.testing.assert_allclose(hs[k][key], ds[key], equal_nan=True, err_msg=f"{k} {key}",
                                           **FLOAT_TOL)
            if p.influence_factor == 0.0:   # the kappa == 0 record skip: the NI share is exactly 0
                assert np.all(hs[k]["neighbor_influence_percent"] == 0.0), k
    finally:
        eng.close()


def test_cfg3_batch_philox_groups_identical():
    """The bench's own stream: the 105-replica batch as one launch per iteration (G=1) and as
    the two concurrent replica groups the bench uses (G=2) give identical lattices and
    records (replica streams are keyed by global replica id, not by group)."""
    _, L, M2, state, reps = bench.workload("cfg3", 0)
    res = {}
    for G in (1, 2):
        eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng="philox", streams=G)
        try:
            assert eng.G == G and eng.tile == (40, 25)
            eng.run(snapshots=False)
            res[G] = ([eng.final_state(k) for k in range(len(reps))], eng.stats_folded().cpu().numpy(),
                      eng.stop_iter.cpu().numpy())
        finally:
            eng.close()
    for a, b in zip(res[1][0], res[2][0]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    assert np.array_equal(res[1][2], res[2][2])
    np.testing.assert_allclose(res[1][1], res[2][1], rtol=1e-12, atol=1e-12)
