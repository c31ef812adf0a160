"""The device MT19937 stream at the layouts the library picks by itself, across chunk boundaries.

The generator splits each replica's draw stream into chains (spgg_mt.h); a chunk is
chains x iterations-per-chain iterations, and at every chunk boundary the chains re-jump
(x^(chunk*W - 1) mod phi) while chain 0 continues from the last chain's key.  A real
SPGG.run crosses hundreds of boundaries (runner.py:88-101: 100,001 iterations).  These runs
use NO layout override (no SPGG_MT_* variables) and go past at least one boundary of the
layout spgg_mt_chains reports; they are checked bit for bit against oracle digests
(tests/golden/mt_layout_digests.json, written by tests/golden/make_mt_layout_golden.py
from oracle/spgg_oracle.py, which tests/golden/*.npz pin to the reference): final S, R, Q,
the whole cooperation-rate history, the C->D switch counts, and the RandomState key after
the run (the reference's draws are algorithms.py:105,108 inside spgg.py:368-592)."""
import hashlib
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from spgg_amd.engine import BatchEngine, ReplicaParams  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mt_layout_digests.json")


def _digest(a, dtype):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=dtype).tobytes()).hexdigest()


@pytest.fixture(autouse=True)
def _no_layout_overrides(monkeypatch):
    for v in ("SPGG_MT_CHAINS", "SPGG_MT_PER_CHAIN", "SPGG_MT_CHUNK", "SPGG_APT", "SPGG_TILE", "SPGG_STREAMS"):
        monkeypatch.delenv(v, raising=False)


@pytest.mark.parametrize("name", ["run100", "cfg3", "cfg5"])
def test_default_layout_across_chunk_boundaries(name):
    case = json.load(open(GOLDEN))[name]
    L, T = case["L"], case["T"]
    reps = [ReplicaParams(**p) for p in case["replica_params"]]
    eng = BatchEngine(L, T, reps, use_second_order=case["M2"], state_representation=case["state"], rng="mt19937")
    try:
        chains, per = case["layout"]
        assert eng.mt_layout == (chains, per), eng.mt_layout
        assert T > chains * per, "the run must cross a chunk boundary"
        eng.run(snapshots=False)
        hs = eng.histories()
        for k, want in case["expected"].items():
            k = int(k)
            Q, R, S = eng.final_state(k)
            assert len(hs[k]["coop_rate_history"]) == len(want["coop_rate_history"]), k
            assert np.array_equal(hs[k]["coop_rate_history"], np.array(want["coop_rate_history"])), k
            assert np.array_equal(hs[k]["switch_C_to_D"], np.array(want["switch_C_to_D"], dtype=np.int64)), k
            assert _digest(S, np.int64) == want["S"], k
            assert _digest(R, np.float64) == want["R"], k
            assert _digest(Q, np.float64) == want["Q"], k
            key, pos = eng.mt_state_host(k)
            assert pos == want["pos"] and _digest(key, np.uint32) == want["key"], k
            assert int(eng.stopped[k]) == want["stop_iter"], k
    finally:
        eng.close()
