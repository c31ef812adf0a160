"""Model of the step kernel's Q write-back bytes per agent-step under write policies / layouts,
from the oracle's trajectories of cfg3 replicas (CPU; a measurement aid, not a test).

The L2 writes a 32-B sector to the fabric if any byte of it is dirty (tools/traffic_calib.hip,
profiles/r06/traffic_calibration.txt: a 16-B store per 32-B sector costs 2x, at a 64-B stride as
well).  Q is held in state planes [s][n][2] (16-B rows), so a sector is 2 agents' rows of one state
(the "sec" columns; they reproduce the measured writes, profiles/r06/traffic/README.txt).  A launch at
iteration t writes, per agent, its TD row (state s_t) and the row its pending NI term of t-1
changed (state s_{t-1}); policies:
  kappa   the NI row is written whenever kappa != 0 (the kernel through round 6)
  nu      only when the NI term is non-zero (max_diff_{t-1} > 0)
  td      TD rows only (an upper bound on what deferring the NI row could give)
  swap    plane 0 holds the row of the agent's current state (a per-agent flag f, swapped -- both
          rows written -- in the launch where s_t != f), plane 1 the other; NI row as "nu"
units: "sec" = a 32-B sector (2 agents of a lattice row: the hardware's write unit), "row" = a 64-B
block (4 agents), "line" = a 128-B line (8 agents: what a line-uniform store policy writes), "2x2" =
a 64-B block of a 2x2 agent block.

    python tools/write_model.py [--t0 6 --t1 25] [--replicas 9]
"""
import argparse
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RUNNER = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
              lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
              reward_weight_payoff=1.0)
L = 200


def blocks(mask, kind):
    """64-B units written: blocks (or half-blocks for "sec") holding at least one marked agent."""
    if kind == "row":
        return int(mask.reshape(L, L // 4, 4).any(axis=2).sum())
    if kind == "line":  # 128-B lines: 8 agents' rows
        return 2 * int(mask.reshape(L, L // 8, 8).any(axis=2).sum())
    if kind == "sec":   # 32-B sectors: 2 agents' rows
        return 0.5 * int(mask.reshape(L, L // 2, 2).any(axis=2).sum())
    return int(mask.reshape(L // 2, 2, L // 2, 2).any(axis=(1, 3)).sum())


def run_one(args):
    r, kappa, seed, t0, t1 = args
    from oracle import spgg_oracle as O
    p = O.Params(L=L, iterations=t1, use_second_order=False, state_representation="reputation",
                 r=r, influence_factor=kappa, **RUNNER)
    prev = {}
    acc = {}
    flag = {}
    extra = {"switchers": 0.0, "nu_nonzero": 0.0}

    def on_step(i, S, R, Q, d):
        s, nu = d["_old_states"], d["_nu"]
        if t0 <= i <= t1 and prev:
            ps, pnu = prev["s"], prev["nu"]
            f = flag.setdefault("f", ps.copy())
            sw = s != f
            ni_other = (ps != s) & (pnu != 0)
            for kind in ("sec", "row", "line", "2x2"):
                n = blocks(np.ones_like(s, dtype=bool), kind) + blocks(sw | ni_other, kind)
                acc[("swap", kind)] = acc.get(("swap", kind), 0.0) + 64.0 * n / (L * L)
            flag["f"] = s.copy()
            for pol in ("kappa", "nu", "td"):
                for kind in ("sec", "row", "line", "2x2"):
                    n = 0
                    for plane in (0, 1):
                        m = s == plane
                        if pol == "kappa" and kappa != 0:
                            m = m | (ps == plane)
                        elif pol == "nu":
                            m = m | ((ps == plane) & (pnu != 0))
                        n += blocks(m, kind)
                    acc[(pol, kind)] = acc.get((pol, kind), 0.0) + 64.0 * n / (L * L)
            extra["switchers"] += float(np.mean(s != ps))
            extra["nu_nonzero"] += float(np.mean(pnu != 0))
        prev["s"], prev["nu"] = s.copy(), nu.copy()

    O.run(p, np.random.RandomState(seed), collect_snapshots=False, on_step=on_step)
    k = t1 - t0 + 1
    return (r, kappa), {key: v / k for key, v in acc.items()}, {key: v / k for key, v in extra.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--t0", type=int, default=6)
    ap.add_argument("--t1", type=int, default=25)
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    jobs = [(r, k, 0, a.t0, a.t1) for r in (2.0, 3.5, 5.0) for k in (0.0, 0.5, 1.0)]
    with ProcessPoolExecutor(a.procs) as ex:
        res = list(ex.map(run_one, jobs))
    keys = [(pol, kind) for pol in ("kappa", "nu", "td", "swap") for kind in ("sec", "row", "line", "2x2")]
    print(f"# Q write-back bytes per agent-step, iterations {a.t0}-{a.t1}, L={L}, seed 0")
    print("%-12s " % "r, kappa" + " ".join("%11s" % f"{p}/{k}" for p, k in keys) + "  switchers  nu!=0")
    for (rk, v, e) in res:
        print("%-12s " % (f"{rk[0]}, {rk[1]}") + " ".join("%11.2f" % v.get(k, 0.0) for k in keys)
              + "  %8.3f  %6.3f" % (e["switchers"], e["nu_nonzero"]))
    print("%-12s " % "mean" + " ".join("%11.2f" % np.mean([v.get(k, 0.0) for _, v, _ in res]) for k in keys))


if __name__ == "__main__":
    main()
