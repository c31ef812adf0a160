"""Golden-fixture helpers shared by the oracle and GPU parity tests.

Fixtures were produced by running the reference itself (tests/golden/make_golden.py).
"""
import glob
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Constructor kwargs the oracle Params understands (spgg.py:50-56).
_PARAM_KEYS = ("r", "c", "cost", "L", "iterations", "alpha", "gamma", "epsilon",
               "epsilon_decay", "epsilon_min", "influence_factor", "use_second_order",
               "lambda_epsilon", "delta_R_D", "R_min", "R_max",
               "reward_weight_payoff", "rep_gain_C", "state_representation", "algorithm")


def case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


class Case:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
        self.meta = json.loads(str(z["meta_json"]))
        self.seed = self.meta["seed"]
        self.kwargs = self.meta["kwargs"]
        self.extra = self.meta["extra"]
        self.datasets = {k[4:]: z[k] for k in z.files if k.startswith("ds__")}
        self.q_table = z["q_table"]
        self.R = z["R"]
        self.Sn = z["Sn"]
        self.ret = z["ret"]
        self.epsilon = float(z["epsilon"])
        self.tables = (z["q_table_1"], z["q_table_2"]) if "q_table_1" in z.files else None

    @property
    def S_in_one(self):
        s = self.extra.get("S_in_one")
        return None if s is None else np.array(s)

    @property
    def algorithm(self):
        from oracle.spgg_oracle import canonical_algorithm
        alg = self.algorithm_instance
        return canonical_algorithm(alg.get("kind", "qlearning") if alg else
                                   self.kwargs.get("algorithm", "qlearning"))

    @property
    def algorithm_instance(self):
        return self.extra.get("algorithm_instance")

    def oracle_params(self):
        from oracle.spgg_oracle import Params
        kw = {k: v for k, v in self.kwargs.items() if k in _PARAM_KEYS}
        p = Params(**kw)
        alg = self.algorithm_instance
        if alg:
            p.algorithm = alg.get("kind", "qlearning")
            p.alg_alpha, p.alg_gamma = alg["alpha"], alg["gamma"]
            p.epsilon, p.epsilon_decay, p.epsilon_min = (
                alg["epsilon"], alg["epsilon_decay"], alg["epsilon_min"])
        return p


def assert_datasets_equal(got, want, exact=True, rtol=1e-5, atol=1e-8, skip=()):
    assert set(got) == set(want), (sorted(set(got) ^ set(want)))
    for k in want:
        if k in skip:
            continue
        g, w = np.asarray(got[k]), np.asarray(want[k])
        assert g.shape == w.shape, (k, g.shape, w.shape)
        if exact or w.dtype.kind in "iub":
            assert np.array_equal(g, w, equal_nan=w.dtype.kind == "f"), k
        else:
            np.testing.assert_allclose(g, w, rtol=rtol, atol=atol, equal_nan=True, err_msg=k)
