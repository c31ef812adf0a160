"""Host logic: the device history record -> reference datasets (CPU only).

The per-step record is synthesised from the oracle's per-agent arrays with the
same sums the kernels accumulate, then `histories_from_stats` must reproduce
the reference's own datasets (golden fixtures)."""
import numpy as np
import pytest

from oracle import spgg_oracle as O
from spgg_amd import _lib as C
from spgg_amd.engine import epsilon_table, histories_from_stats
from tests._golden import Case, assert_datasets_equal, case_names

EXACT = {"coop_rate_history", "switch_C_to_D", "switch_D_to_C", "epsilon_history_final",
         "best_neighbor_second_order_percent"} | {f"group_comp_d{d}_history" for d in range(6)}


def record_from_oracle(c):
    p = c.oracle_params()
    L, n = p.L, p.L * p.L
    T = p.iterations
    st = np.zeros((T + 2, C.NSTAT))
    rs = np.random.RandomState(c.seed)
    Q, tables = O.init_tables(p, rs)
    S = rs.randint(0, 2, size=(L, L)) if c.S_in_one is None else c.S_in_one
    R = np.zeros((L, L))
    eps = p.epsilon
    st[1, C.ST_NCOOP] = np.sum(S == 0)
    last, stopped = 0, False
    for i in range(1, T + 1):
        P = O.payoff(S, p)
        st[i, C.ST_SUMP] = P.sum()
        st[i, C.ST_SUMP_C] = P[S == 0].sum()
        st[i, C.ST_SUMP_D] = P[S == 1].sum()
        st[i, C.ST_SUMR] = R.sum()
        last = i
        nc = np.sum(S == 0)
        if nc == 0 or nc == n:
            stopped = True
            break
        draws = O.draw_step(rs, L, p.algorithm)
        S, R, Q, d = O.step(S, R, Q, eps, draws, p=p, P=P, tables=tables)
        eps = max(eps * p.epsilon_decay, p.epsilon_min)
        a, ps = d["_actions"], d["_prev_S"]
        rew, rr = d["_rewards"], d["_rep_reward"]
        st[i + 1, C.ST_NCOOP] = np.sum(a == 0)
        st[i, C.ST_SW_CD] = d["switch_C_to_D"]
        st[i, C.ST_SW_DC] = d["switch_D_to_C"]
        st[i, C.ST_SUM_WPP] = (p.reward_weight_payoff * d["_P"]).sum()
        st[i, C.ST_SUM_WRR] = (p.reward_weight_rep * rr).sum()
        st[i, C.ST_SUM_REW_C] = rew[a == 0].sum()
        st[i, C.ST_SUM_REW_D] = rew[a == 1].sum()
        wr = p.reward_weight_rep * rr
        st[i, C.ST_SUM_RATIO_C] = ((np.abs(wr) / (np.abs(rew) + 1e-9)) * 100)[a == 0].sum()
        nd = O.sum5((a == 1).astype(int))
        for k in range(6):
            st[i, C.ST_GC0 + k] = np.sum(nd == k)
        md, mi = d["_max_diff"], d["_max_idx"]
        st[i, C.ST_NMD_POS] = np.sum(md > 0)
        st[i, C.ST_NMD_POS2] = np.sum((md > 0) & (mi >= 4))
        nu = d["_nu"]
        st[i, C.ST_SUM_PCT] = (np.abs(nu) / (d["_atd2"] + np.abs(nu) + 1e-8) * 100).sum()
        for e in range(4):
            qv = Q[:, :, e // 2, e % 2]
            st[i, C.ST_SUMQ + e] = qv.sum()
            st[i, C.ST_SUMQ_C + e] = qv[ps == 0].sum()
            st[i, C.ST_SUMQ_D + e] = qv[ps == 1].sum()
    return st, last, stopped, epsilon_table(p.epsilon, p.epsilon_decay, p.epsilon_min, T + 1), n


@pytest.mark.parametrize("name", case_names())
def test_histories_from_record_match_reference(name):
    c = Case(name)
    st, last, stopped, eps, n = record_from_oracle(c)
    got = histories_from_stats(st, last, stopped, eps, n)
    want = {k: v for k, v in c.datasets.items() if k in got}
    assert set(got) == set(want)
    for k in want:
        g, w = got[k], want[k]
        assert g.shape == w.shape and g.dtype == w.dtype or (g.size == 0 and w.size == 0), k
        if k in EXACT:
            assert np.array_equal(g, w, equal_nan=True), k
        else:
            np.testing.assert_allclose(g, w, rtol=1e-12, atol=1e-15, equal_nan=True, err_msg=k)
