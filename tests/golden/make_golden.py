"""Generate golden vectors by running the REFERENCE itself (survey container only).

    python tests/golden/make_golden.py  [--ref /root/reference]

The reference (`src/model/spgg.py`) imports `h5py` at module top; h5py is not
installed, so an in-memory stand-in records every `create_dataset` call.
`SPGG.__init__` reseeds the global MT19937 from OS entropy (spgg.py:98); the
seed is pinned by making a no-argument `numpy.random.seed()` seed a fixed value.

Each case is written to `tests/golden/<name>.npz`:
  meta_json  — constructor kwargs + seed (JSON string)
  ds__<name> — every dataset the reference's run() wrote (the layout manifest)
  q_table, R, Sn, ret, epsilon — state after run()
Only these data files travel; the reference never leaves this container.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# (name, seed, constructor kwargs).  Runner-style defaults (runner.py:88-101)
# unless the case says otherwise.
RUNNER = dict(c=1, cost=1, num_of_strategies=2, K=0.1, population_type=0,
              alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99,
              epsilon_min=0.01, lambda_epsilon=0.01, delta_R_C=1, delta_R_D=1,
              R_min=-10, R_max=10, rep_gain_C=1.0)

CASES = [
    ("m1_rep_L16", 0, dict(RUNNER, r=3.0, L=16, iterations=200, influence_factor=1.0,
                           use_second_order=False, reward_weight_payoff=0.95,
                           state_representation="reputation")),
    ("m2_act_L16", 1, dict(RUNNER, r=3.6, L=16, iterations=200, influence_factor=0.5,
                           use_second_order=True, reward_weight_payoff=1.0,
                           state_representation="action")),
    ("m2_rep_L24_stopC", 0, dict(RUNNER, r=5.0, L=24, iterations=800, influence_factor=1.0,
                                 use_second_order=True, reward_weight_payoff=0.95,
                                 state_representation="reputation")),
    ("m1_rep_L24_stopD", 0, dict(RUNNER, r=1.0, L=24, iterations=650, influence_factor=1.0,
                                 use_second_order=False, reward_weight_payoff=0.95,
                                 state_representation="reputation")),
    ("m1_act_L20_k0", 2, dict(RUNNER, r=2.0, L=20, iterations=150, influence_factor=0.0,
                              use_second_order=False, reward_weight_payoff=0.95,
                              state_representation="action")),
    ("m1_rep_L50_cfg1", 0, dict(RUNNER, r=3.0, L=50, iterations=300, influence_factor=1.0,
                                use_second_order=False, reward_weight_payoff=0.95,
                                state_representation="reputation")),
    ("m2_rep_L18_wp083", 2, dict(RUNNER, r=4.0, L=18, iterations=200, influence_factor=0.0,
                                 use_second_order=True, reward_weight_payoff=0.83,
                                 state_representation="reputation")),
    ("defaults_L12", 3, dict(L=12, iterations=120)),  # SPGG's own defaults (spgg.py:50-56)
    ("m1_rep_L16_k2", 4, dict(RUNNER, r=3.6, L=16, iterations=120, influence_factor=2.0,
                              use_second_order=False, reward_weight_payoff=1.0,
                              state_representation="reputation")),
    ("m1_rep_L10_snap", 5, dict(RUNNER, r=3.8, L=10, iterations=1001, influence_factor=1.0,
                                use_second_order=False, reward_weight_payoff=0.95,
                                state_representation="reputation")),
    ("m2_act_L13_odd", 6, dict(RUNNER, r=3.0, L=13, iterations=150, influence_factor=1.0,
                               use_second_order=True, reward_weight_payoff=0.95,
                               state_representation="action")),
] + [
    (f"step{k}_m1_rep_L16", 7, dict(RUNNER, r=3.0, L=16, iterations=k, influence_factor=1.0,
                                    use_second_order=False, reward_weight_payoff=0.95,
                                    state_representation="reputation"))
    for k in (1, 2, 3)
] + [
    (f"step{k}_m2_rep_L16", 8, dict(RUNNER, r=3.0, L=16, iterations=k, influence_factor=1.0,
                                    use_second_order=True, reward_weight_payoff=0.95,
                                    state_representation="reputation"))
    for k in (1, 2, 3)
]

# The other three operators of algorithms.py:136-341 (SARSA draws three times
# per step, Double-Q keeps two tables and draws an extra rand per step).
CASES += [
    ("sarsa_m1_rep_L16", 20, dict(RUNNER, r=3.0, L=16, iterations=200, influence_factor=1.0,
                                  use_second_order=False, reward_weight_payoff=0.95,
                                  state_representation="reputation", algorithm="sarsa")),
    ("sarsa_m2_act_L14", 21, dict(RUNNER, r=3.6, L=14, iterations=150, influence_factor=0.5,
                                  use_second_order=True, reward_weight_payoff=1.0,
                                  state_representation="action", algorithm="sarsa")),
    ("esarsa_m1_rep_L16", 22, dict(RUNNER, r=3.0, L=16, iterations=200, influence_factor=1.0,
                                   use_second_order=False, reward_weight_payoff=0.95,
                                   state_representation="reputation", algorithm="expected_sarsa")),
    ("esarsa_m2_rep_L18", 23, dict(RUNNER, r=4.2, L=18, iterations=150, influence_factor=1.5,
                                   use_second_order=True, reward_weight_payoff=0.9,
                                   state_representation="reputation", algorithm="expected-sarsa")),
    ("dq_m1_rep_L16", 24, dict(RUNNER, r=3.0, L=16, iterations=200, influence_factor=1.0,
                               use_second_order=False, reward_weight_payoff=0.95,
                               state_representation="reputation", algorithm="double_qlearning")),
    ("dq_m2_act_L15", 25, dict(RUNNER, r=3.8, L=15, iterations=150, influence_factor=1.0,
                               use_second_order=True, reward_weight_payoff=1.0,
                               state_representation="action", algorithm="double-q-learning")),
    ("dq_m1_rep_L24_stopD", 26, dict(RUNNER, r=1.0, L=24, iterations=700, influence_factor=1.0,
                                     use_second_order=False, reward_weight_payoff=0.95,
                                     state_representation="reputation", algorithm="double_qlearning")),
    ("sarsa_m2_rep_L20_stopC", 27, dict(RUNNER, r=5.0, L=20, iterations=800, influence_factor=1.0,
                                        use_second_order=True, reward_weight_payoff=0.95,
                                        state_representation="reputation", algorithm="sarsa")),
]

# Lattices smaller than the stencils (L < 5: the M=2 offsets wrap onto the same
# cells several times; L=1: every neighbour is the agent itself, absorbed at t=1).
CASES += [
    ("tiny_m1_rep_L1", 41, dict(RUNNER, r=3.0, L=1, iterations=20, influence_factor=1.0,
                                use_second_order=False, reward_weight_payoff=0.95,
                                state_representation="reputation")),
    ("tiny_m2_rep_L2", 42, dict(RUNNER, r=3.6, L=2, iterations=60, influence_factor=1.0,
                                use_second_order=True, reward_weight_payoff=0.95,
                                state_representation="reputation")),
    ("tiny_m2_rep_L3", 43, dict(RUNNER, r=4.0, L=3, iterations=80, influence_factor=1.0,
                                use_second_order=True, reward_weight_payoff=0.95,
                                state_representation="reputation")),
    ("tiny_m1_act_L4", 44, dict(RUNNER, r=3.0, L=4, iterations=80, influence_factor=0.5,
                                use_second_order=False, reward_weight_payoff=1.0,
                                state_representation="action")),
    ("tiny_m2_act_L5", 45, dict(RUNNER, r=3.8, L=5, iterations=80, influence_factor=1.0,
                                use_second_order=True, reward_weight_payoff=0.95,
                                state_representation="action")),
    ("tiny_dq_m2_rep_L3", 46, dict(RUNNER, r=4.0, L=3, iterations=60, influence_factor=1.0,
                                   use_second_order=True, reward_weight_payoff=0.95,
                                   state_representation="reputation", algorithm="double_qlearning")),
    ("tiny_sarsa_m1_rep_L6", 47, dict(RUNNER, r=3.6, L=6, iterations=80, influence_factor=1.0,
                                      use_second_order=False, reward_weight_payoff=0.95,
                                      state_representation="reputation", algorithm="sarsa")),
]

# Cases that need objects (S_in_one, an algorithm instance) are built below.
SPECIAL = ["sinone_L16", "algo_instance_L16", "absorbing_init_L8",
           "sarsa_instance_L16", "esarsa_instance_L16", "dq_instance_L16"]


class _FakeH5File:
    def __init__(self, fn, mode="r"):
        self.fn, self.mode, self.data = fn, mode, {}
        _FakeH5File.last = self

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def create_dataset(self, name, data=None):
        self.data[name] = np.array(data)


def _import_reference(ref):
    import matplotlib
    matplotlib.use("Agg")
    sys.modules["h5py"] = types.SimpleNamespace(File=_FakeH5File)
    sys.path.insert(0, ref)
    from src.model import SPGG, QLearning, SARSA, ExpectedSARSA, DoubleQLearning  # noqa: E402
    return SPGG, dict(qlearning=QLearning, sarsa=SARSA, expected_sarsa=ExpectedSARSA,
                      double_qlearning=DoubleQLearning)


def _pin_seed(seed):
    orig = np.random.seed

    def seed_fn(s=None):
        orig(seed if s is None else s)
    np.random.seed = seed_fn
    return orig


def _run(SPGG, seed, kwargs, tmp):
    orig = _pin_seed(seed)
    try:
        m = SPGG(**kwargs)
    finally:
        np.random.seed = orig
    m.folder = tmp
    ret = m.run(os.path.join(tmp, "x.h5"))
    return m, ret, _FakeH5File.last.data


def _save(name, seed, kwargs, m, ret, data, extra=None):
    out = {"meta_json": np.array(json.dumps(dict(seed=seed, kwargs=kwargs, extra=extra or {})))}
    for k, v in data.items():
        out["ds__" + k] = v
    out["q_table"] = m.q_table
    out["R"] = m.R
    out["Sn"] = np.asarray(m._Sn)
    out["ret"] = np.array([float(x) for x in ret])
    out["epsilon"] = np.array(m.algorithm.epsilon)
    if getattr(m.algorithm, "q_table_1", None) is not None:   # Double-Q's two tables
        out["q_table_1"] = m.algorithm.q_table_1
        out["q_table_2"] = m.algorithm.q_table_2
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated name prefixes to (re)generate")
    args = ap.parse_args()
    SPGG, ALGS = _import_reference(args.ref)
    QLearning = ALGS["qlearning"]
    only = [x for x in args.only.split(",") if x]

    def want(name):
        return not only or any(name.startswith(o) for o in only)

    with tempfile.TemporaryDirectory() as tmp:
        for name, seed, kw in CASES:
            if not want(name):
                continue
            m, ret, data = _run(SPGG, seed, kw, tmp)
            _save(name, seed, kw, m, ret, data)
            print(name, "iters", len(data["coop_rate_history"]), "coop", ret[0])

        # algorithm instances of the other operators, with their own hyper-parameters
        for name, seed, kind, m2, state in (("sarsa_instance_L16", 30, "sarsa", True, "reputation"),
                                            ("esarsa_instance_L16", 31, "expected_sarsa", False, "action"),
                                            ("dq_instance_L16", 32, "double_qlearning", True, "reputation")):
            if not want(name):
                continue
            alg = dict(alpha=0.6, gamma=0.85, epsilon=0.4, epsilon_decay=0.97, epsilon_min=0.02)
            kw = dict(RUNNER, r=3.4, L=16, iterations=120, influence_factor=1.0,
                      use_second_order=m2, reward_weight_payoff=0.95, state_representation=state)
            m, ret, data = _run(SPGG, seed, dict(kw, algorithm=ALGS[kind](**alg)), tmp)
            _save(name, seed, kw, m, ret, data, extra={"algorithm_instance": dict(alg, kind=kind)})
            print(name, "iters", len(data["coop_rate_history"]), "coop", ret[0])
        if only and not any(want(n) for n in ("sinone_L16", "algo_instance_L16", "absorbing_init_L8")):
            return

        # S_in_one supplied: no population draw (spgg.py:161-162)
        rs = np.random.RandomState(99)
        S0 = rs.randint(0, 2, size=(16, 16))
        kw = dict(RUNNER, r=3.0, L=16, iterations=100, influence_factor=1.0,
                  use_second_order=False, reward_weight_payoff=0.95)
        m, ret, data = _run(SPGG, 11, dict(kw, S_in_one=S0), tmp)
        _save("sinone_L16", 11, kw, m, ret, data, extra={"S_in_one": S0.tolist()})

        # algorithm instance whose alpha/gamma/epsilon differ from SPGG's (spgg.py:115-116)
        alg = dict(alpha=0.5, gamma=0.8, epsilon=0.3, epsilon_decay=0.98, epsilon_min=0.05)
        kw = dict(RUNNER, r=3.4, L=16, iterations=100, influence_factor=1.0,
                  use_second_order=True, reward_weight_payoff=0.95)
        m, ret, data = _run(SPGG, 12, dict(kw, algorithm=QLearning(**alg)), tmp)
        _save("algo_instance_L16", 12, kw, m, ret, data, extra={"algorithm_instance": alg})

        # absorbing initial population: stop at iteration 1, no step draws
        S0 = np.zeros((8, 8), dtype=int)
        kw = dict(RUNNER, r=3.0, L=8, iterations=50)
        m, ret, data = _run(SPGG, 13, dict(kw, S_in_one=S0), tmp)
        _save("absorbing_init_L8", 13, kw, m, ret, data, extra={"S_in_one": S0.tolist()})


if __name__ == "__main__":
    main()
