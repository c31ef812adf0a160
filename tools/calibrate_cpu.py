"""Calibrate the CPU baseline: the oracle (oracle/spgg_oracle.py, the NumPy restatement
bench.py times on the GPU box) against the reference's own SPGG.run, same workload, same
core, same process.  Survey container only (the reference never travels).

    python tools/calibrate_cpu.py [--ref /root/reference] [--out profiles/r03/cpu_calibration.json]

Workload: BASELINE.json configs[1] / cfg2 -- L=200, r=3.0, kappa=1.0, M=1, reputation
state, w_P=0.95, the runner's constants (runner.py:88-101).  Steady per-iteration cost =
(time of a 210-iteration run - time of a 110-iteration run) / 100: both runs include the
same construction, snapshot (iterations 1, 10, 100: PNG + histogram) and epilogue costs,
so the difference is 100 plain iterations (iterations 111-210).  One thread
(OMP/MKL/OPENBLAS_NUM_THREADS=1), medians over --repeats interleaved pairs.
"""
import argparse
import json
import os
import platform
import sys
import tempfile
import time

for v in ("OMP_NUM_THREADS", "MKL_NUM_THREADS", "OPENBLAS_NUM_THREADS"):
    os.environ[v] = "1"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from tests.golden import make_golden as G  # noqa: E402  (reference import helpers)
from oracle import spgg_oracle as O  # noqa: E402

KW = dict(G.RUNNER, r=3.0, L=200, influence_factor=1.0, use_second_order=False,
          reward_weight_payoff=0.95, state_representation="reputation")


def time_reference(SPGG, T, seed=0):
    with tempfile.TemporaryDirectory() as tmp:
        t0 = time.perf_counter()
        G._run(SPGG, seed, dict(KW, iterations=T), tmp)
        return time.perf_counter() - t0


def time_oracle(T, seed=0):
    p = O.Params(L=KW["L"], iterations=T, use_second_order=False, state_representation="reputation",
                 **{k: KW[k] for k in ("r", "c", "cost", "alpha", "gamma", "epsilon", "epsilon_decay",
                                       "epsilon_min", "influence_factor", "lambda_epsilon", "delta_R_D",
                                       "R_min", "R_max", "reward_weight_payoff", "rep_gain_C")})
    t0 = time.perf_counter()
    O.run(p, np.random.RandomState(seed), collect_snapshots=True)
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03", "cpu_calibration.json"))
    ap.add_argument("--repeats", type=int, default=7)
    args = ap.parse_args()
    SPGG, _ = G._import_reference(args.ref)
    # interleaved (reference, oracle) pairs: the container's virtual CPU drifts by tens of %
    fns = (("reference", lambda T: time_reference(SPGG, T)), ("oracle", time_oracle))
    steps = {"reference": [], "oracle": []}
    for _ in range(args.repeats):
        for name, fn in fns:
            a, b = fn(110), fn(210)
            steps[name].append((b - a) / 100)
    ratios = sorted(r / o for r, o in zip(steps["reference"], steps["oracle"]))
    res = {k: float(np.median(v)) for k, v in steps.items()}
    for k, v in steps.items():
        print(f"{k}: median {res[k] * 1e3:.2f} ms/iteration ({', '.join(f'{s * 1e3:.2f}' for s in v)})", flush=True)
    n = KW["L"] ** 2
    out = {
        "workload": "cfg2: L=200 r=3.0 kappa=1.0 M=1 reputation w_P=0.95, runner constants",
        "method": ("(t(210 iterations) - t(110 iterations)) / 100, one thread, %d interleaved "
                   "(reference, oracle) pairs; medians" % args.repeats),
        "reference_ms_per_iteration": res["reference"] * 1e3,
        "oracle_ms_per_iteration": res["oracle"] * 1e3,
        "reference_ms_samples": [x * 1e3 for x in steps["reference"]],
        "oracle_ms_samples": [x * 1e3 for x in steps["oracle"]],
        "reference_agent_steps_per_s": n / res["reference"],
        "oracle_agent_steps_per_s": n / res["oracle"],
        "oracle_over_reference": float(np.median(ratios)),
        "oracle_over_reference_range": [ratios[0], ratios[-1]],
        "cpu": platform.processor() or platform.machine(),
        "numpy": np.__version__,
        "python": platform.python_version(),
    }
    try:
        with open("/proc/cpuinfo") as f:
            out["cpu"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
