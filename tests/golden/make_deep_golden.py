"""Digest of one runner-shaped run of the REFERENCE deep into its snapshot schedule.

    python tests/golden/make_deep_golden.py [--ref /root/reference]   (survey container only)

One `SPGG(L=100, iterations=10001, ...)` with the runner's constants
(src/experiments/runner.py:88-101), seed pinned as in make_golden.py, so the run
passes the snapshot iterations 5000 and 10000 (spgg.py:153,397-402) and the extra
PNG at 5000 (spgg.py:553).  10,001 iterations of an L=100 lattice are too large to
commit as arrays, so `deep_L100_10001.json` holds:
  exact   -- sha256 of every dataset compared bit for bit (the integer datasets, the
             snapshots, the cooperation-rate / switch / group-composition histories,
             the final state) and of q_table, R, _Sn, the return tuple and the global
             MT19937 key the run leaves behind;
  approx  -- the device-reduced float histories (tests/test_gpu_parity.py APPROX)
             every 10th value plus the full-length sum, for the 1e-5 comparison.
Only this data file travels; the reference never leaves this container.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import tempfile

import numpy as np

import make_golden as G

HERE = os.path.dirname(os.path.abspath(__file__))
NAME = "deep_L100_10001"
SEED = 3
KWARGS = dict(G.RUNNER, r=3.6, L=100, iterations=10001, influence_factor=1.0, use_second_order=False,
              reward_weight_payoff=0.95, state_representation="reputation")
STRIDE = 10

APPROX = {"it_records_final", "rep_avg_history_final", "neighbor_influence_percent",
          "payoff_component_history", "rep_component_history", "reputation_reward_ratio",
          "avg_reward_C_history", "avg_reward_D_history"} | {
    f"{g}_q_{s}_{a}_history" for g in ("cooperators", "defectors", "avg")
    for s in ("s0", "s1") for a in ("c", "d")}


def digest(a) -> dict:
    """dtype, shape and sha256 of an array's C-order bytes (the comparison key)."""
    a = np.ascontiguousarray(np.asarray(a))
    return {"dtype": a.dtype.str, "shape": list(a.shape), "sha256": hashlib.sha256(a.tobytes()).hexdigest()}


def approx_record(a) -> dict:
    a = np.asarray(a, dtype=np.float64)
    flat = a.reshape(a.shape[0], -1) if a.ndim > 1 else a
    return {"shape": list(a.shape), "stride": STRIDE,
            "values": np.where(np.isnan(flat[::STRIDE]), None, flat[::STRIDE]).tolist(),
            "nansum": np.nansum(flat, axis=0).tolist(), "nan_count": int(np.isnan(flat).sum())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    SPGG, _ = G._import_reference(args.ref)
    with tempfile.TemporaryDirectory() as tmp:
        m, ret, data = G._run(SPGG, SEED, KWARGS, tmp)
        pngs = sorted(os.listdir(os.path.join(tmp, "plots", "snapshots"))) \
            if os.path.isdir(os.path.join(tmp, "plots", "snapshots")) else []
    out = {"meta": {"seed": SEED, "kwargs": KWARGS, "generator": "tests/golden/make_deep_golden.py",
                    "iterations_recorded": int(len(data["coop_rate_history"])), "png": pngs},
           "exact": {}, "approx": {}}
    for k, v in sorted(data.items()):
        if k in APPROX:
            out["approx"][k] = approx_record(v)
        else:
            out["exact"][k] = digest(v)
    out["exact"]["__q_table"] = digest(m.q_table)
    out["exact"]["__R"] = digest(m.R)
    out["exact"]["__Sn"] = digest(np.asarray(m._Sn))
    out["exact"]["__ret"] = digest(np.array([float(x) for x in ret]))
    out["meta"]["ret"] = [float(x) for x in ret]
    out["meta"]["epsilon"] = float(m.algorithm.epsilon)
    st = np.random.get_state()   # the global MT19937 key the run leaves (the drop-in restores it)
    out["exact"]["__mt_key"] = digest(np.asarray(st[1], dtype=np.uint32))
    out["meta"]["mt_pos"] = int(st[2])
    with open(os.path.join(HERE, NAME + ".json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(NAME, "iterations", out["meta"]["iterations_recorded"], "ret", ret, "png", pngs)


if __name__ == "__main__":
    main()
