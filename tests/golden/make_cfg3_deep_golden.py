"""Oracle digests of 1,000 iterations of three cfg3 replicas -- the depth the headline kernel
instance runs at (eps reaches eps_min at t ~ 390, so most of these iterations are the steady
regime a 10,000-iteration run lives in).

    python tests/golden/make_cfg3_deep_golden.py        (~2 minutes of CPU here, 3 processes)

Replicas: bench.py's cfg3 grid at r = 3.5 (i = 3), kappa = 0, 0.5, 1 (one of each: the
recomputed NI record is off, on at half strength and on), seed 0, w_P = 1.0.  Recorded per
replica from oracle/spgg_oracle.py (pinned bit-exactly to the reference by tests/golden/*.npz):
SHA-256 of the final S (int64), R (float64), Q (float64, (L,L,2,2)) and of the RandomState key
after the run (uint32[624]) and its pos, the executed iteration count, the exact histories
(cooperation rate, switches, group composition) and the float histories the kernels accumulate
(NI percent, Q means, rewards, reputation), checked within 1e-5 (north_star).  GPU side:
tests/test_gpu_cfg3_deep.py.  Data only: nothing of the reference travels.
"""
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

OUT = os.path.join(HERE, "cfg3_deep_digests.json")
L, T = 200, 1000
RUNNER = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
              lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
              reward_weight_payoff=1.0, influence_factor=1.0, r=3.5)
REPLICAS = [dict(RUNNER, influence_factor=k, seed=0) for k in (0.0, 0.5, 1.0)]
EXACT = ("coop_rate_history", "switch_C_to_D", "switch_D_to_C") + tuple(f"group_comp_d{d}_history" for d in range(6))
FLOAT = ("neighbor_influence_percent", "avg_q_s0_c_history", "avg_q_s1_d_history", "cooperators_q_s0_c_history",
         "defectors_q_s1_d_history", "rep_avg_history_final", "avg_reward_C_history", "avg_reward_D_history",
         "payoff_component_history", "rep_component_history")


def digest(a, dtype):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=dtype).tobytes()).hexdigest()


def run_one(p):
    from oracle import spgg_oracle as O
    p = dict(p)
    seed = p.pop("seed")
    op = O.Params(L=L, iterations=T, use_second_order=False, state_representation="reputation", **p)
    rs = np.random.RandomState(seed)
    ds, fin = O.run(op, rs, collect_snapshots=False)
    st = rs.get_state()
    out = {"S": digest(fin["S"], np.int64), "R": digest(fin["R"], np.float64), "Q": digest(fin["Q"], np.float64),
           "key": digest(st[1], np.uint32), "pos": int(st[2]), "stop_iter": int(fin["stop_iter"])}
    for k in EXACT + FLOAT:   # (JSON floats round-trip exactly: the exact keys compare bit for bit)
        out[k] = [float(x) for x in np.asarray(ds[k]).reshape(-1)]
    return out


def main():
    t0 = time.time()
    with ProcessPoolExecutor(len(REPLICAS)) as ex:
        res = list(ex.map(run_one, REPLICAS))
    doc = {"L": L, "T": T, "replica_params": REPLICAS, "exact": list(EXACT), "float": list(FLOAT), "expected": res}
    with open(OUT, "w") as f:
        json.dump(doc, f)
    print(f"wrote {OUT} ({time.time() - t0:.0f} s): executed", [len(r["coop_rate_history"]) for r in res])


if __name__ == "__main__":
    main()
