"""The operator interface called directly (host NumPy path of spgg_amd.algorithms) against
single calls of the REFERENCE's own operators (tests/golden/operator_calls.npz, made by
tests/golden/make_operator_golden.py): outputs, the updated tables and the position of the
global np.random stream after the call, bit for bit (algorithms.py:102-341)."""
import json
import os

import numpy as np
import pytest

from spgg_amd import algorithms as A

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "operator_calls.npz")
_Z = np.load(GOLD)
_META = json.loads(str(_Z["meta_json"]))
_KINDS = dict(qlearning=A.QLearning, sarsa=A.SARSA, expected_sarsa=A.ExpectedSARSA,
              double_qlearning=A.DoubleQLearning)


@pytest.mark.parametrize("case", _META["cases"], ids=lambda c: f"{c['kind']}-{c['call']}-L{c['L']}")
def test_operator_call_matches_reference(case):
    tag, L = case["tag"], case["L"]
    x = {k.split("__in_")[1]: _Z[k] for k in _Z.files if k.startswith(tag + "__in_")}
    alg = _KINDS[case["kind"]](**_META["hyper"])
    if case["kind"] == "double_qlearning" and case["call"] != "select":
        alg.q_table_1, alg.q_table_2 = x["t1"].copy(), x["t2"].copy()
    np.random.seed(case["seed"])
    q = x["q"].copy()
    if case["call"].startswith("select"):
        res = alg.select_action(q, x["s"], L)
    else:
        kw = dict(next_actions=x["a2"]) if case["kind"] == "sarsa" else {}
        res = alg.update_q_table(q, x["s"], x["a"], x["r"], x["s2"], **kw)
    after = np.random.rand()
    want = _Z[tag + "__result"]
    assert res.dtype == want.dtype and np.array_equal(res, want)
    assert np.array_equal(q, _Z[tag + "__q_after"])          # in place, as the reference's
    assert after == float(_Z[tag + "__rand_after"])             # the same draws consumed
    if tag + "__t1_after" in _Z.files:
        assert np.array_equal(alg.q_table_1, _Z[tag + "__t1_after"])
        assert np.array_equal(alg.q_table_2, _Z[tag + "__t2_after"])


def test_operator_errors_match_reference():
    """The reference's ValueErrors: SARSA without next_actions (algorithms.py:159-160), Double Q
    before initialize_q_tables (:300-301)."""
    q = np.zeros((3, 3, 2, 2))
    z = np.zeros((3, 3), dtype=int)
    with pytest.raises(ValueError, match="SARSA requires 'next_actions' parameter"):
        A.SARSA(0.1, 0.9, 0.5, 0.99, 0.01).update_q_table(q, z, z, np.zeros((3, 3)), z)
    with pytest.raises(ValueError, match="Q-tables not initialized"):
        A.DoubleQLearning(0.1, 0.9, 0.5, 0.99, 0.01).update_q_table(q, z, z, np.zeros((3, 3)), z)
    with pytest.raises(NotImplementedError):
        A.RLAlgorithm(0.1, 0.9, 0.5, 0.99, 0.01).update_q_table(q, z, z, np.zeros((3, 3)), z)


def test_builtin_operators_still_run_on_the_device_path():
    """Giving the classes host methods does not make them 'custom': SPGG.run keeps fusing the
    four built-in operators into the HIP step (operator_kind), and a subclass that redefines a
    method is still refused."""
    for kind, cls in _KINDS.items():
        assert A.operator_kind(cls(**_META["hyper"])) == kind

    class Custom(A.QLearning):
        def update_q_table(self, q_table, old_states, actions, rewards, new_states, **kwargs):
            return q_table
    with pytest.raises(ValueError, match="Custom.*update_q_table"):
        A.operator_kind(Custom(**_META["hyper"]))
