"""Pipeline properties of the HIP path on the GPU: shard invariance of a sharded sweep, the
generator's ordering after the caller's stream, and the generator's error path.

* Shard invariance: the reference fans a sweep out over a process
  pool (/root/reference/src/experiments/runner.py:136-154); here a sweep is sharded over ranks
  as contiguous replica blocks (distributed.run_sharded: BatchEngine(replica_offset=...)).  A
  replica's results must not depend on the shard it lands in: the Philox stream is keyed by
  the GLOBAL replica id, the MT19937 stream by the replica's own seed (its chain layout is
  chosen from the shard's batch size).
* Ordering: a run's first generator chunks read mt_state / eps / stop_iter, which the caller
  may write on its own stream just before spgg_step; the generator waits for that stream.
* Error path: a generator wait that exhausted its bound sets the context's error word;
  spgg_status reports it without a sync, spgg_flush fails with SPGG_E_STATE, and the engine
  raises instead of returning a silently wrong run."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from spgg_amd import _lib as C  # noqa: E402
from spgg_amd.engine import BatchEngine, ReplicaParams  # noqa: E402
from oracle import spgg_oracle as O  # noqa: E402

RUNNER = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
              lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
              reward_weight_payoff=0.95, influence_factor=1.0, r=3.0)


def _reps(n):
    return [ReplicaParams(**dict(RUNNER, r=2.5 + 0.25 * (k % 7), influence_factor=0.5 * (k % 3), seed=300 + k))
            for k in range(n)]


def _results(eng):
    return ([eng.final_state(k) for k in range(eng.R)], eng.stats_folded().cpu().numpy(),
            eng.stop_iter.cpu().numpy(), eng.mt_state.cpu().numpy())


@pytest.mark.parametrize("rng,L,T", [("philox", 200, 40), ("mt19937", 200, 40), ("philox", 48, 150)])
def test_sharded_batch_equals_whole_batch(rng, L, T):
    """A 12-replica batch run whole, and as the two shards run_sharded builds for a world of 2
    (replicas 0-5 at replica_offset 0, 6-11 at replica_offset 6): bit-identical per-replica
    lattices, Q tables, absorbing stops, history records and (MT19937) keys."""
    reps = _reps(12)
    whole = BatchEngine(L, T, reps, use_second_order=False, rng=rng)
    try:
        whole.run(snapshots=False)
        want = _results(whole)
    finally:
        whole.close()
    got = []
    for off in (0, 6):
        eng = BatchEngine(L, T, reps[off:off + 6], use_second_order=False, rng=rng, replica_offset=off)
        try:
            eng.run(snapshots=False)
            got.append(_results(eng))
        finally:
            eng.close()
    for half, off in zip(got, (0, 6)):
        for k in range(6):
            for x, y in zip(half[0][k], want[0][off + k]):
                assert np.array_equal(x, y), (rng, off + k)
        # history records: f64 atomics of the workgroups, added in launch order: equal to rounding
        np.testing.assert_allclose(half[1], want[1][off:off + 6], rtol=1e-12, atol=1e-12)
        assert np.array_equal(half[2], want[2][off:off + 6]), rng
        if rng == "mt19937":
            assert np.array_equal(half[3], want[3][off:off + 6]), rng


def test_generator_waits_for_the_callers_stream():
    """The key is written on torch's stream behind a ~50 ms device spin, immediately before
    the run: the generator (a non-blocking stream for a batch this small) must still read the
    key the copy writes, so the run equals the oracle's."""
    L, T = 40, 60
    p = ReplicaParams(**dict(RUNNER, seed=11))
    eng = BatchEngine(L, T, [p], use_second_order=False, rng="mt19937")
    try:
        good = eng.mt_state.clone()
        eng.mt_state.fill_(0x5A5A5A5A)             # a wrong key in place ...
        torch.cuda.synchronize()
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(100_000_000)         # ... a long device spin on torch's stream ...
        else:
            a = torch.rand(4096, 4096, dtype=torch.float64, device=eng.dev)
            for _ in range(4):
                a = a @ a / 4096
        eng.mt_state.copy_(good)                   # ... then the real key, in stream order
        eng.run(snapshots=False)                   # (no host sync before the first chunk)
        op = O.Params(L=L, iterations=T, use_second_order=False, state_representation="reputation",
                      **{k: getattr(p, k) for k in ("r", "c", "cost", "alpha", "gamma", "epsilon", "epsilon_decay",
                                                     "epsilon_min", "influence_factor", "lambda_epsilon",
                                                     "delta_R_D", "R_min", "R_max", "reward_weight_payoff",
                                                     "rep_gain_C")})
        rs = np.random.RandomState(11)
        ds, fin = O.run(op, rs, collect_snapshots=False)
        Q, R, S = eng.final_state(0)
        assert np.array_equal(S, fin["S"]) and np.array_equal(R, fin["R"]) and np.array_equal(Q, fin["Q"])
        key, pos = eng.mt_state_host(0)
        st = rs.get_state()
        assert pos == st[2] and np.array_equal(key, st[1])
    finally:
        eng.close()


def test_generator_error_word_fails_the_run():
    """spgg_test_set_error ORs SPGG_GEN_ERR_SPIN into the word as an exhausted wait does:
    spgg_status reports it, spgg_flush returns SPGG_E_STATE with a message, and BatchEngine
    raises at its next host check instead of finishing with wrong draws."""
    L, T = 32, 40
    eng = BatchEngine(L, T, [ReplicaParams(**dict(RUNNER, seed=5))], use_second_order=False, rng="mt19937")
    try:
        g = eng.groups[0]
        f = ctypes.c_uint32()
        eng.step(5)
        torch.cuda.synchronize()
        C.check(eng.lib.spgg_status(g["ctx"], ctypes.byref(f)), g["ctx"], "spgg_status")
        assert f.value == 0
        C.check(eng.lib.spgg_test_set_error(g["ctx"], C.GEN_ERR_SPIN), g["ctx"], "spgg_test_set_error")
        rc = eng.lib.spgg_flush(g["ctx"], 5, ctypes.c_void_p(eng.stream))
        assert rc == C.E_STATE, rc
        assert b"generator" in eng.lib.spgg_last_error(g["ctx"])
        C.check(eng.lib.spgg_status(g["ctx"], ctypes.byref(f)), g["ctx"], "spgg_status")
        assert f.value == C.GEN_ERR_SPIN
        with pytest.raises(C.SpggError, match="generator"):
            eng.check_status()
    finally:
        eng.close()


def test_philox_context_reports_no_generator_error():
    eng = BatchEngine(24, 5, [ReplicaParams(**dict(RUNNER, seed=1))], use_second_order=False, rng="philox")
    try:
        f = ctypes.c_uint32(7)
        C.check(eng.lib.spgg_status(eng.ctx, ctypes.byref(f)), eng.ctx, "spgg_status")
        assert f.value == 0
        eng.run(snapshots=False)
    finally:
        eng.close()
