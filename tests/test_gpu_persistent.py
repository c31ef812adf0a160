"""Persistent launches (spgg_persist_kernel, spgg_persistent) against the per-launch path and the
oracle.

A batch whose tiles all fit the device at once runs each spgg_step call (MT19937: each generator
chunk of it) as ONE launch: the workgroups keep their agents' Q rows in registers across the
iterations and meet at a per-replica barrier instead of a launch boundary (the lattice max and
NCOOP, src/model/spgg.py:405,488, and the neighbours' halos; sc1 hand-offs).  Results must not
change: S, R, Q, the absorbing iterations, snapshots and the MT19937 keys bit-identical to the
per-launch path (SPGG_PERSIST=0) over >= 300 iterations, the history records equal up to the
order of the f64 atomics, and the workloads checked against the oracle."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from spgg_amd.engine import BatchEngine, ReplicaParams  # noqa: E402

FLOAT_TOL = dict(rtol=1e-5, atol=1e-9)


def _params(**kw):
    base = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
                lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
                reward_weight_payoff=0.95, influence_factor=1.0, r=3.0)
    base.update(kw)
    return ReplicaParams(**base)


def _run(monkeypatch, persist, L, T, reps, M2=False, state="reputation", rng="philox", alg="qlearning",
         snapshots=False, chunk=256):
    monkeypatch.setenv("SPGG_PERSIST", "1" if persist else "0")
    eng = BatchEngine(L, T, reps, use_second_order=M2, state_representation=state, rng=rng, algorithm=alg)
    try:
        assert eng.persistent == persist, (eng.persistent, eng.persist_capacity, eng.tile)
        eng.run(chunk=chunk, snapshots=snapshots)
        out = dict(final=[eng.final_state(k) for k in range(len(reps))],
                   stats=eng.stats_folded().cpu().numpy(), stop=eng.stop_iter.cpu().numpy().copy(),
                   mt=eng.mt_state.cpu().numpy().copy(), snaps=[dict(s) for s in eng.snapshots],
                   hist=eng.histories())
        if alg == "double_qlearning":
            out["tables"] = [eng.final_tables(k) for k in range(len(reps))]
        return out
    finally:
        eng.close()


def _same(a, b):
    for x, y in zip(a["final"], b["final"]):
        for u, v in zip(x, y):
            assert np.array_equal(u, v)
    assert np.array_equal(a["stop"], b["stop"])
    assert np.array_equal(a["mt"], b["mt"])
    for sa, sb in zip(a["snaps"], b["snaps"]):
        assert sa.keys() == sb.keys()
        for k in sa:
            for u, v in zip(sa[k], sb[k]):
                assert np.array_equal(np.asarray(u), np.asarray(v))
    for ha, hb in zip(a["hist"], b["hist"]):
        for k in ha:
            x, y = np.asarray(ha[k]), np.asarray(hb[k])
            if x.dtype.kind in "iub":
                assert np.array_equal(x, y), k
            else:   # (sums of f64 atomics in another order: equal to rounding)
                np.testing.assert_allclose(x, y, rtol=1e-12, atol=1e-12, err_msg=k)
    if "tables" in a:
        for x, y in zip(a["tables"], b["tables"]):
            for u, v in zip(x, y):
                assert np.array_equal(u, v)


@pytest.mark.parametrize("shape", ["cfg5", "cfg4", "cfg2_mt", "absorbing"])
def test_persistent_matches_per_launch(shape, monkeypatch):
    """>= 300 iterations of each shape, persistent vs one launch per iteration: identical state,
    stops, snapshots and keys.  cfg5: one L=1000 replica, 1000 tiles over the 8 XCDs (16
    barrier shards); cfg4: 8 x L=200 M=2 action (two replica groups, both persistent at once);
    cfg2_mt: L=200 on the device MT19937 stream across generator chunks, run() with its
    snapshot stops; absorbing: replicas that absorb at C and at D mid-launch beside live ones."""
    if shape == "cfg5":
        kw = dict(L=1000, T=300, reps=[_params(r=3.6, seed=5)])
    elif shape == "cfg4":
        kw = dict(L=200, T=300, reps=[_params(seed=s) for s in range(8)], M2=True, state="action")
    elif shape == "cfg2_mt":
        kw = dict(L=200, T=1001, reps=[_params(seed=2)], rng="mt19937", snapshots=True)
    else:
        # (eps decays to 0, so the lattice can absorb: at eps_min = 0.01 some of its 3600 agents
        # explore every iteration)
        fast = dict(epsilon_decay=0.95, epsilon_min=0.0)
        # (the oracle: r = 1.0 seed 7 absorbs at t = 170, r = 0.6 seed 12 at t = 161; the others run on)
        kw = dict(L=60, T=1500, reps=[_params(r=1.0, seed=7, **fast), _params(r=5.0, seed=8, **fast),
                                     _params(r=3.4, seed=9), _params(r=1.0, influence_factor=0.0, seed=10, **fast),
                                     _params(r=0.6, seed=12, **fast)],
                  chunk=300, rng="mt19937")
    a = _run(monkeypatch, True, **kw)
    b = _run(monkeypatch, False, **kw)
    if shape == "absorbing":   # stops inside persistent launches, at the oracle's iterations
        assert list(a["stop"]) == [170, 0, 0, 0, 161], a["stop"]
    _same(a, b)


@pytest.mark.parametrize("alg", ["sarsa", "expected_sarsa"])
@pytest.mark.parametrize("M2,state", [(False, "reputation"), (True, "action")])
def test_persistent_operators_match_per_launch(alg, M2, state, monkeypatch):
    """SARSA (which keeps the stored pending NI record: carried in registers across a persistent
    launch) and Expected SARSA on the device MT19937 stream.  (Double Q's 512-agent tiles at
    L=200 are 25 x 20, a run-time width: no persistent instance, one launch per iteration --
    test_persistent_plan_by_batch_size.)"""
    kw = dict(L=200, T=300, reps=[_params(seed=s, r=3.0 + 0.4 * s) for s in range(3)], M2=M2, state=state,
              rng="mt19937", alg=alg)
    _same(_run(monkeypatch, True, **kw), _run(monkeypatch, False, **kw))


def test_persistent_cfg2_mt19937_vs_oracle(monkeypatch):
    """The persistent path against the oracle itself: L=200, 400 iterations on the device MT19937
    stream (two generator chunks), S / R / Q and the exact histories bit for bit."""
    from oracle import spgg_oracle as O
    p = _params(seed=3)
    monkeypatch.setenv("SPGG_PERSIST", "1")
    eng = BatchEngine(200, 400, [p], use_second_order=False, rng="mt19937")
    assert eng.persistent
    eng.run(snapshots=False)
    Q, R, S = eng.final_state(0)
    h = eng.histories()[0]
    eng.close()
    op = O.Params(L=200, iterations=400, r=p.r, c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5,
                  epsilon_decay=0.99, epsilon_min=0.01, influence_factor=1.0, use_second_order=False,
                  lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, reward_weight_payoff=0.95,
                  rep_gain_C=1.0)
    ds, fin = O.run(op, np.random.RandomState(3), collect_snapshots=False)
    assert np.array_equal(S, fin["S"]) and np.array_equal(R, fin["R"]) and np.array_equal(Q, fin["Q"])
    assert np.array_equal(h["coop_rate_history"], ds["coop_rate_history"])
    np.testing.assert_allclose(h["neighbor_influence_percent"], ds["neighbor_influence_percent"], **FLOAT_TOL)


def test_persistent_plan_by_batch_size(monkeypatch):
    """Persistent exactly when the whole batch's tiles fit the device at once: cfg5 (1000 tiles),
    cfg4 (8 x 80) and cfg2 do; cfg3 (105 replicas x 40 tiles) does not (with SPGG_PERSIST=1; the
    default is one launch per iteration)."""
    monkeypatch.setenv("SPGG_PERSIST", "1")
    for L, n, M2, state, want in ((1000, 1, False, "reputation", True), (200, 8, True, "action", True),
                                  (200, 1, False, "reputation", True), (200, 105, False, "reputation", False)):
        eng = BatchEngine(L, 2, [_params(seed=s) for s in range(n)], use_second_order=M2,
                          state_representation=state, rng="philox")
        try:
            tiles = n * (L // eng.tile[0]) * (-(-L // eng.tile[1]))
            assert eng.persistent == want, (L, n, eng.tile, eng.persist_capacity)
            assert eng.persistent == (tiles <= eng.persist_capacity)
        finally:
            eng.close()
    # no persistent instance for run-time-width tiles (Double Q at L=200: 25 x 20 or, one replica, 25 x 10)
    eng = BatchEngine(200, 2, [_params(seed=0)], use_second_order=False, rng="philox", algorithm="double_qlearning")
    try:
        assert eng.tile[0] not in (20, 40) and not eng.persistent and eng.persist_capacity == 0, eng.tile
    finally:
        eng.close()
