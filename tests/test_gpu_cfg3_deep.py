"""The headline kernel instance through 1,000 iterations against oracle digests.

cfg3's batch runs spgg_step_kernel at four agents per thread on 40 x 25 tiles with the
recomputed pending NI record (spgg_kernels.hip, RECOMP), one launch per iteration.  Elsewhere
that instance is checked against the oracle only to t = 300, while eps reaches eps_min at t ~ 390
and a 10,000-iteration run spends > 96 % of its iterations past it.  Three of cfg3's replicas
(r = 3.5, kappa = 0 / 0.5 / 1, seed 0: tests/golden/cfg3_deep_digests.json, written by
tests/golden/make_cfg3_deep_golden.py from the oracle) are stepped here 1,000 iterations on the
device MT19937 stream with that instance forced (SPGG_APT=max: a 3-replica batch would otherwise
take two agents per thread; the second case runs the same replicas in persistent launches,
SPGG_PERSIST=1): final S, R, Q, the RandomState key after the run and the exact histories bit for bit,
the float histories within 1e-5 (north_star).  Reference: spgg.py:368-592 (the loop body),
477-509 (the NI record the kernel recomputes)."""
import hashlib
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from spgg_amd.engine import BatchEngine, ReplicaParams  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg3_deep_digests.json")


def _digest(a, dtype):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=dtype).tobytes()).hexdigest()


@pytest.mark.parametrize("mode", ["headline_instance", "persistent"])
def test_cfg3_replicas_1000_iterations_vs_oracle(mode, monkeypatch):
    case = json.load(open(GOLDEN))
    L, T = case["L"], case["T"]
    for v in ("SPGG_MT_CHAINS", "SPGG_MT_PER_CHAIN", "SPGG_MT_CHUNK", "SPGG_TILE", "SPGG_STREAMS"):
        monkeypatch.delenv(v, raising=False)
    if mode == "headline_instance":
        monkeypatch.setenv("SPGG_APT", "max")
        monkeypatch.setenv("SPGG_PERSIST", "0")
    else:
        monkeypatch.delenv("SPGG_APT", raising=False)
        monkeypatch.setenv("SPGG_PERSIST", "1")
    reps = [ReplicaParams(**p) for p in case["replica_params"]]
    eng = BatchEngine(L, T, reps, use_second_order=False, rng="mt19937")
    try:
        if mode == "headline_instance":
            assert eng.tile == (40, 25) and not eng.persistent, (eng.tile, eng.persistent)
        else:
            assert eng.persistent, (eng.tile, eng.persist_capacity)
        eng.run(snapshots=False)
        hs = eng.histories()
        for k, want in enumerate(case["expected"]):
            Q, R, S = eng.final_state(k)
            assert int(eng.stopped[k]) == want["stop_iter"], k
            for key in case["exact"]:
                assert np.array_equal(np.asarray(hs[k][key], dtype=np.float64).reshape(-1),
                                      np.asarray(want[key], dtype=np.float64)), (k, key)
            for key in case["float"]:
                np.testing.assert_allclose(np.asarray(hs[k][key], dtype=np.float64).reshape(-1),
                                           np.asarray(want[key]), rtol=1e-5, atol=1e-9, err_msg=f"{k} {key}")
            assert _digest(S, np.int64) == want["S"], k
            assert _digest(R, np.float64) == want["R"], k
            assert _digest(Q, np.float64) == want["Q"], k
            key, pos = eng.mt_state_host(k)
            assert pos == want["pos"] and _digest(key, np.uint32) == want["key"], k
    finally:
        eng.close()
