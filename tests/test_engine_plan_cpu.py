"""Replica-group / cache-wave planning of BatchEngine (engine.plan_groups): pure host
arithmetic, checked against the configurations measured on the MI355X."""
import pytest

from spgg_amd.engine import plan_groups

MB = 2 ** 20
BUDGET = 240 * MB


def per_rep(L, qw=4, rsz=1):  # engine.state_bytes_per_replica for Q-learning, int8 reputation
    return int(L * L * (qw * 8 + 8 + 4 + 2 + 2 * rsz) * 1.1)


@pytest.mark.parametrize("R,L,want", [
    (105, 200, (1, 2, 2)),     # cfg3: fits the cache, 2 groups of 2100 workgroups
    (52, 200, (1, 3, 3)),      # 2080 tiles: 3 groups
    (35, 200, (1, 3, 3)),
    (1, 200, (1, 1, 1)),       # cfg2
    (8, 200, (1, 2, 2)),       # cfg4-sized batch (320 tiles): two groups
    (16, 200, (1, 2, 2)),
    (4, 200, (1, 1, 1)),       # 160 tiles: one group
    (126, 200, (2, 4, 2)),     # past the cache: 2 waves of 2 resident groups
    (210, 200, (2, 4, 2)),
    (420, 200, (4, 8, 2)),     # 4 waves of cfg3-sized work
    (1, 1000, (1, 1, 1)),      # cfg5
    (8, 1000, (2, 4, 2)),
    (3000, 50, (2, 4, 2)),     # many small lattices
])
def test_auto_plan(R, L, want):
    assert plan_groups(R, L, per_rep(L), BUDGET) == want


def test_waves_never_exceed_replicas_and_groups_never_exceed_replicas():
    for R in (1, 2, 3, 7, 50):
        w, g, r = plan_groups(R, 4000, per_rep(4000), BUDGET)   # one replica alone exceeds the cache
        assert 1 <= w <= R and 1 <= g <= R and 1 <= r <= g


def test_explicit_streams_and_single():
    assert plan_groups(105, 200, per_rep(200), BUDGET, streams=6) == (1, 6, 6)
    assert plan_groups(105, 200, per_rep(200), BUDGET, streams=500) == (1, 105, 105)
    w, g, r = plan_groups(105, 200, per_rep(200), 80 * MB, streams=6)
    assert (w, g, r) == (3, 6, 2)
    assert plan_groups(420, 200, per_rep(200), BUDGET, single=True) == (1, 1, 1)


def test_resident_groups_fit_the_budget():
    for R in (126, 150, 210, 315, 420, 1000):
        w, g, r = plan_groups(R, 200, per_rep(200), BUDGET)
        assert r * -(-R // g) * per_rep(200) <= BUDGET * 1.05, (R, w, g, r)


@pytest.mark.parametrize("double_q", [False, True])
def test_state_plane_layout_round_trip(double_q):
    """The Q buffer's state planes (spgg_abi.h): plane s holds every agent's row s, and the
    conversion back gives the reference's (L, L, 2, 2) table(s) bit for bit."""
    import numpy as np
    from spgg_amd.engine import from_state_planes, to_state_planes
    L = 5
    rs = np.random.RandomState(3)
    tabs = [rs.uniform(-0.01, 0.01, size=(L, L, 2, 2)) for _ in range(2 if double_q else 1)]
    buf = to_state_planes(*tabs)
    assert buf.shape == (2, L * L, 4 if double_q else 2)
    y, x, s = 3, 1, 1
    assert np.array_equal(buf[s, y * L + x, :2], tabs[0][y, x, s])
    if double_q:
        assert np.array_equal(buf[s, y * L + x, 2:], tabs[1][y, x, s])
    back = from_state_planes(buf.reshape(-1), L, double_q)
    assert len(back) == len(tabs)
    for a, b in zip(back, tabs):
        assert np.array_equal(a, b)
