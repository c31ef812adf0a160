"""Golden vectors of single RL-operator calls, made by running the REFERENCE's own
operator classes (survey container only; src/model/algorithms.py imports numpy alone, so
the module is loaded from its file without the package __init__, which needs h5py).

    python tests/golden/make_operator_golden.py  [--ref /root/reference]

Cases (written to tests/golden/operator_calls.npz, one key prefix per case):
  * select_action of all four operators (Double-Q with and without its tables);
  * update_q_table of Q-learning, SARSA (next_actions passed), Expected SARSA, Double Q;
  * each call from a pinned global seed, with the first rand() drawn AFTER the call
    (the stream position the call left: rand then randint per select, Double-Q's table draw).
Inputs are recorded beside the outputs; only this data file travels.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "operator_calls.npz")

HYPER = dict(alpha=0.7, gamma=0.85, epsilon=0.35, epsilon_decay=0.99, epsilon_min=0.01)


def _load(ref):
    spec = importlib.util.spec_from_file_location("ref_algorithms", os.path.join(ref, "src", "model",
                                                                                 "algorithms.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _inputs(L, seed):
    rs = np.random.RandomState(1000 + seed)
    q = rs.uniform(-1.0, 1.0, size=(L, L, 2, 2))
    q[0, 0, 0, :] = 0.25            # a tie: argmax -> action 0
    q[1 % L, 0, 1, :] = -0.5
    return dict(q=q, s=rs.randint(0, 2, size=(L, L)), a=rs.randint(0, 2, size=(L, L)),
                r=rs.uniform(-0.2, 1.2, size=(L, L)), s2=rs.randint(0, 2, size=(L, L)),
                a2=rs.randint(0, 2, size=(L, L)),
                t1=rs.uniform(-0.01, 0.01, size=(L, L, 2, 2)), t2=rs.uniform(-0.01, 0.01, size=(L, L, 2, 2)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    A = _load(args.ref)
    kinds = dict(qlearning=A.QLearning, sarsa=A.SARSA, expected_sarsa=A.ExpectedSARSA,
                 double_qlearning=A.DoubleQLearning)
    out, cases = {}, []
    k = 0
    for L in (5, 12):
        for name, cls in kinds.items():
            for call in ("select", "update") + (("select_tables",) if name == "double_qlearning" else ()):
                k += 1
                x = _inputs(L, k)
                alg = cls(**HYPER)
                if name == "double_qlearning" and call != "select":
                    alg.q_table_1, alg.q_table_2 = x["t1"].copy(), x["t2"].copy()
                np.random.seed(k)
                q = x["q"].copy()
                if call.startswith("select"):
                    res = alg.select_action(q, x["s"], L)
                else:
                    kw = dict(next_actions=x["a2"]) if name == "sarsa" else {}
                    res = alg.update_q_table(q, x["s"], x["a"], x["r"], x["s2"], **kw)
                after = np.random.rand()
                tag = f"c{k}"
                cases.append(dict(tag=tag, L=L, kind=name, call=call, seed=k))
                for key, v in x.items():
                    out[f"{tag}__in_{key}"] = v
                out[f"{tag}__result"] = np.asarray(res)
                out[f"{tag}__q_after"] = q
                out[f"{tag}__rand_after"] = np.array(after)
                if name == "double_qlearning" and alg.q_table_1 is not None:
                    out[f"{tag}__t1_after"] = alg.q_table_1
                    out[f"{tag}__t2_after"] = alg.q_table_2
    out["meta_json"] = np.array(json.dumps(dict(hyper=HYPER, cases=cases)))
    np.savez_compressed(OUT, **out)
    print(f"{len(cases)} operator calls -> {OUT}")


if __name__ == "__main__":
    main()
