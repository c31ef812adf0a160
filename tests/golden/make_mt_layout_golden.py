"""Oracle digests of long runs at the library's DEFAULT MT19937 chain layouts.

    python tests/golden/make_mt_layout_golden.py          (~5 minutes of CPU here)

The device generator splits a replica's draw stream into chains (spgg_mt.h); a chunk is
chains x iterations-per-chain iterations and every chunk boundary re-jumps the chains.
These cases run past at least one boundary of the layout `choose_mt_chains` picks for
them (asserted by tests/test_gpu_mt_layouts.py through spgg_mt_chains):

  run100  L=100, runner constants, T=1200          layout  8 x 34 (272-iteration chunks)
  cfg3    the 105-replica bench batch, T=300        layout  4 x 32 (128), 4 replicas checked
  cfg5    L=1000, r=3.6, T=260                      layout 256 x 1 (256)

Recorded per replica, from oracle/spgg_oracle.py (itself pinned bit-exactly to the
reference by tests/golden/*.npz): SHA-256 of the final S (int64), R (float64), Q (float64,
(L,L,2,2)), of the RandomState key after the run (uint32[624]) and its pos, the whole
coop_rate_history and switch_C_to_D (small), and the executed iteration count.  The GPU
test compares the device run's bytes with these digests (bit-exact).  Data only: nothing
of the reference travels.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

OUT = os.path.join(HERE, "mt_layout_digests.json")

RUNNER = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
              lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
              reward_weight_payoff=0.95, influence_factor=1.0, r=3.0)

# cfg3 replica k = i*15 + j*5 + s: r = 2.0 + 0.5 i, kappa = (0, 0.5, 1)[j], seed s (bench.workload);
# both replica groups (0-52, 53-104) and all three kappas appear
CFG3_CHECKED = (41, 57, 63, 99)


def digest(a, dtype):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=dtype).tobytes()).hexdigest()


def cases():
    out = {"run100": dict(L=100, T=1200, M2=False, state="reputation", layout=[8, 34],
                          replicas=[dict(RUNNER, seed=0)], checked=[0])}
    cfg3 = [dict(RUNNER, r=2.0 + 0.5 * i, influence_factor=k, reward_weight_payoff=1.0, seed=s)
            for i in range(7) for k in (0.0, 0.5, 1.0) for s in range(5)]
    out["cfg3"] = dict(L=200, T=300, M2=False, state="reputation", layout=[4, 32], replicas=cfg3,
                       checked=list(CFG3_CHECKED))
    out["cfg5"] = dict(L=1000, T=260, M2=False, state="reputation", layout=[256, 1],
                       replicas=[dict(RUNNER, r=3.6, seed=0)], checked=[0])
    return out


def run_case(c, k):
    from oracle import spgg_oracle as O
    p = dict(c["replicas"][k])
    seed = p.pop("seed")
    op = O.Params(L=c["L"], iterations=c["T"], use_second_order=c["M2"], state_representation=c["state"], **p)
    rs = np.random.RandomState(seed)
    ds, fin = O.run(op, rs, collect_snapshots=False)
    st = rs.get_state()
    return {"S": digest(fin["S"], np.int64), "R": digest(fin["R"], np.float64), "Q": digest(fin["Q"], np.float64),
            "key": digest(st[1], np.uint32), "pos": int(st[2]), "stop_iter": int(fin["stop_iter"]),
            "coop_rate_history": [float(x) for x in ds["coop_rate_history"]],
            "switch_C_to_D": [int(x) for x in ds["switch_C_to_D"]]}


def main():
    res = {}
    for name, c in cases().items():
        t0 = time.time()
        res[name] = {key: c[key] for key in ("L", "T", "M2", "state", "layout", "checked")}
        res[name]["replica_params"] = c["replicas"]
        res[name]["expected"] = {str(k): run_case(c, k) for k in c["checked"]}
        n = [len(v["coop_rate_history"]) for v in res[name]["expected"].values()]
        print(f"{name}: executed {n} iterations ({time.time() - t0:.0f} s)", flush=True)
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
