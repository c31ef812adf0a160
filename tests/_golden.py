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


# fixtures that are not whole reference runs (single operator calls: test_operator_host_cpu.py)
NOT_RUNS = {"operator_calls"}


def case_names():
    return sorted(n for n in (os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))
                  if n not in NOT_RUNS)


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


class DeepDigest:
    """A deep run of the reference (tests/golden/make_deep_golden.py): sha256 digests of the
    datasets compared bit for bit, every 10th value + the sums of the float histories."""

    def __init__(self, name="deep_L100_10001"):
        with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
            d = json.load(f)
        self.meta, self.exact, self.approx = d["meta"], d["exact"], d["approx"]
        self.seed, self.kwargs = self.meta["seed"], self.meta["kwargs"]

    @staticmethod
    def digest(a):
        import hashlib
        a = np.ascontiguousarray(np.asarray(a))
        return {"dtype": a.dtype.str, "shape": list(a.shape),
                "sha256": hashlib.sha256(a.tobytes()).hexdigest()}

    def check(self, datasets, q_table, R, Sn, ret, rtol=1e-5, atol=1e-9, mt_key=None):
        """Assert a run's datasets and final state match: exact ones by digest (dtype, shape,
        bytes), float histories at every 10th value and by their sums within rtol."""
        finals_names = {"__q_table", "__R", "__Sn", "__ret", "__mt_key"}
        want_names = set(self.exact) - finals_names | set(self.approx)
        assert set(datasets) == want_names, sorted(set(datasets) ^ want_names)
        finals = {"__q_table": q_table, "__R": R, "__Sn": np.asarray(Sn),
                  "__ret": np.array([float(x) for x in ret])}
        if mt_key is not None:
            finals["__mt_key"] = np.asarray(mt_key, dtype=np.uint32)
        for k, w in self.exact.items():
            if k == "__mt_key" and mt_key is None:
                continue
            g = self.digest(finals[k] if k in finals else datasets[k])
            assert g == w, (k, g["dtype"], g["shape"], w["dtype"], w["shape"])
        for k, w in self.approx.items():
            a = np.asarray(datasets[k], dtype=np.float64)
            assert list(a.shape) == w["shape"], (k, a.shape, w["shape"])
            flat = a.reshape(a.shape[0], -1) if a.ndim > 1 else a
            vals = np.array([np.nan if v is None else v for v in
                             (np.ravel(w["values"]) if flat.ndim == 1 else
                              [x for row in w["values"] for x in row])], dtype=np.float64)
            np.testing.assert_allclose(flat[::w["stride"]].reshape(-1), vals, rtol=rtol, atol=atol,
                                       equal_nan=True, err_msg=k)
            np.testing.assert_allclose(np.nansum(flat, axis=0), np.array(w["nansum"]), rtol=rtol,
                                       atol=atol * flat.shape[0], err_msg=k + " (sum)")
            assert int(np.isnan(flat).sum()) == w["nan_count"], k
