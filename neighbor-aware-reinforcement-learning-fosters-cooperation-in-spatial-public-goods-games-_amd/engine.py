"""Batched replica engine: many independent SPGG lattices stepped on one MI355X.

Host side of the hot path.  It owns the device buffers (torch tensors used only
as HBM allocations), fills the per-replica parameter table with constants
computed in the reference's own Python-float arithmetic, and drives
`libspgg_hip.so` through its C ABI (`include/spgg_abi.h`).  The per-step
history record each replica accumulates on the device is turned back into the
reference's HDF5 datasets (`src/model/spgg.py:594-633`) by `histories()`.

Random streams:
  * "mt19937": init draws on the host exactly as SPGG.__init__ does
    (spgg.py:121-127,162) from `numpy.random.RandomState`; the continuing
    MT19937 key is moved to the device, which draws every step's rand(L,L)
    and randint(0,2,(L,L)) (algorithms.py:105,108) -- plus SARSA's two
    further selects and Double-Q's table choice -- bit-identically.
  * "inject": the host draws each step (tests / debugging).
  * "philox": counter-based Philox2x32-10 stream (one block per agent pair and
    iteration); statistical parity only.
"""
from __future__ import annotations

import atexit
import ctypes
import dataclasses
import math
import os
from typing import Callable, Optional, Sequence

import numpy as np
import torch

from . import _lib as C
from .algorithms import canonical_name

SNAPSHOT_ITERS = (1, 10, 100, 1000, 5000, 10000, 20000, 30000, 40000)  # spgg.py:153


def tuning_env(name: str, default: Optional[str] = None) -> Optional[str]:
    """A scheduling / layout knob (SPGG_CACHE_MB, SPGG_CHUNK, SPGG_STREAMS, ...), read only when
    SPGG_TUNING=1 -- as the library reads its own (spgg_abi.h, "Environment knobs"): a stray
    variable in a user's environment never changes how a production run is scheduled."""
    if os.environ.get("SPGG_TUNING") != "1":
        return default
    return os.environ.get(name, default)
PNG_ITERS = set(SNAPSHOT_ITERS) | {5000}                                 # spgg.py:553


@dataclasses.dataclass
class ReplicaParams:
    """Constructor arguments of one replica (spgg.py:50-56 + the RL operator's own)."""
    r: float = 2
    c: float = 1
    cost: float = 0.5
    alpha: float = 0.1            # SPGG.alpha (diagnostic TD / NI percent, spgg.py:475)
    gamma: float = 0.9            # SPGG.gamma (diagnostic TD, spgg.py:473)
    epsilon: float = 0.5          # operator's eps schedule (algorithms.py:40-42)
    epsilon_decay: float = 0.995
    epsilon_min: float = 0.01
    influence_factor: float = 1.0
    lambda_epsilon: float = 0.01
    delta_R_D: float = 1
    R_min: float = -10
    R_max: float = 10
    reward_weight_payoff: float = 1.0
    rep_gain_C: float = 0.5
    alg_alpha: Optional[float] = None  # operator's alpha if it differs (algorithm instance)
    alg_gamma: Optional[float] = None
    seed: Optional[int] = None         # RandomState seed (mt19937/inject) or Philox key

    def to_c(self) -> C.RepParams:
        p = C.RepParams()
        r, c = self.r, self.c
        p.rc = float(r * c)                              # spgg.py:256 (r*c first)
        p.cost = float(self.cost)
        norm_max, norm_min = 4 * r, r - 5                # spgg.py:148-149
        p.norm_min = float(norm_min)
        p.norm_den = float(norm_max - norm_min)          # spgg.py:377
        p.norm_rcp = 1.0 / p.norm_den                    # correctly rounded (device: Markstein)
        p.w_p = float(self.reward_weight_payoff)
        p.w_rep = float(1 - self.reward_weight_payoff)   # spgg.py:108
        p.alpha = float(self.alpha if self.alg_alpha is None else self.alg_alpha)
        p.gamma = float(self.gamma if self.alg_gamma is None else self.alg_gamma)
        p.diag_alpha = float(self.alpha)
        p.diag_gamma = float(self.gamma)
        p.kappa = float(self.influence_factor)
        p.lambda_eps = float(self.lambda_epsilon)
        p.rep_gain_c = float(self.rep_gain_C)
        p.neg_delta_r_d = float(-self.delta_R_D)
        p.r_min = float(self.R_min)
        p.r_max = float(self.R_max)
        p.seed = int(self.seed or 0) & 0xFFFFFFFFFFFFFFFF
        rc = r * c
        for N in range(6):                               # spgg.py:256-257, N cooperators
            tk = rc * N / 5
            p.pay_c[N] = float(tk - self.cost)
            p.pay_d[N] = float(tk)
        u = self.rep_unit()
        if u is not None:
            p.rep_unit = u
            p.rk_gain = int(self.rep_gain_C / u)
            p.rk_loss = int(self.delta_R_D / u)
            p.rk_min = int(self.R_min / u)
            p.rk_max = int(self.R_max / u)
        return p

    def rep_unit(self):
        """Dyadic unit u (1, 1/2, ..., 1/1024) such that rep_gain_C, delta_R_D,
        R_min, R_max are exact multiples of u with every reachable R/u in int8,
        or None.  Then R = k*u exactly for every R the reference produces
        (R starts at 0, spgg.py:129; updates spgg.py:321-323 stay exact), so
        the int8 lattice reproduces the f64 one bit for bit."""
        vals = [self.rep_gain_C, self.delta_R_D, self.R_min, self.R_max]
        try:
            vals = [float(v) for v in vals]
        except (TypeError, ValueError):
            return None
        if not all(math.isfinite(v) for v in vals) or vals[2] > vals[3] or vals[2] > 0 or vals[3] < 0:
            return None
        for m in range(11):
            u = 2.0 ** -m
            ks = [v / u for v in vals]
            if all(k == int(k) for k in ks):
                g, l_, lo, hi = (int(k) for k in ks)
                if -128 <= lo and hi <= 127 and abs(g) <= 127 and abs(l_) <= 127:
                    return u
                return None
        return None


def to_state_planes(*tables) -> np.ndarray:
    """One replica's Q buffer (spgg_abi.h) from its (L, L, 2, 2) table(s): plane s holds every
    agent's row s -- (2, n, 2), or for Double-Q's two tables (2, n, 4) with q_table_1's row
    then q_table_2's -- so a launch writes back only the rows it changed."""
    rows = [np.asarray(t, dtype=np.float64).reshape(-1, 2, 2) for t in tables]   # (n, s, a)
    return np.stack([np.concatenate([r[:, s, :] for r in rows], axis=1) for s in range(2)])


def from_state_planes(buf: np.ndarray, L: int, double_q: bool = False):
    """The (L, L, 2, 2) table(s) of one replica's Q buffer (inverse of to_state_planes)."""
    planes = np.asarray(buf).reshape(2, L * L, 4 if double_q else 2)
    tabs = [np.ascontiguousarray(planes[:, :, 2 * i:2 * i + 2].transpose(1, 0, 2)).reshape(L, L, 2, 2)
            for i in range(2 if double_q else 1)]
    return tuple(tabs)


def epsilon_table(eps0, decay, emin, n):
    """eps in effect at iterations 1..n (index t), decayed after every step (algorithms.py:42)."""
    out = np.empty(n + 1)
    out[0] = eps0
    e = eps0
    for t in range(1, n + 1):
        out[t] = e
        e = max(e * decay, emin)
    return out


@dataclasses.dataclass
class InitState:
    Q: np.ndarray                 # (L, L, 2, 2) float64
    S: np.ndarray                 # (L, L) int
    tables: Optional[tuple] = None       # Double-Q: (q_table_1, q_table_2), each (L, L, 2, 2)
    mt_key: Optional[np.ndarray] = None  # (624,) uint32 continuing MT19937 key
    mt_pos: int = 0
    rs: Optional[np.random.RandomState] = None  # host stream (inject mode)


def reference_init(L: int, rs: np.random.RandomState, S_in_one=None, algorithm="qlearning") -> InitState:
    """SPGG.__init__'s draws: Q ~ U(-0.01, 0.01) (spgg.py:121), for Double-Q two
    more tables whose mean replaces Q (spgg.py:124-127, algorithms.py:250-266),
    then S ~ randint(0,2) (spgg.py:162)."""
    Q = rs.uniform(low=-0.01, high=0.01, size=(L, L, 2, 2))
    tables = None
    if canonical_name(algorithm) == "double_qlearning":
        q1 = rs.uniform(low=-0.01, high=0.01, size=(L, L, 2, 2))
        q2 = rs.uniform(low=-0.01, high=0.01, size=(L, L, 2, 2))
        tables, Q = (q1, q2), (q1 + q2) / 2
    S = rs.randint(0, 2, size=(L, L)) if S_in_one is None else np.asarray(S_in_one)
    st = rs.get_state()
    return InitState(Q=Q, S=S, tables=tables, mt_key=np.asarray(st[1], dtype=np.uint32),
                     mt_pos=int(st[2]), rs=rs)


def plan_groups(R: int, L: int, bytes_per_replica: int, cache_bytes: int, streams: Optional[int] = None,
                single: bool = False):
    """(waves, groups, resident) for a batch of R replicas of an L x L lattice.

    Replica groups run on concurrent HIP streams, so one group's launch tail overlaps
    another's start.  Groups per wave by the wave's 1000-agent tiles (measured on
    MI355X, profiles/r02/streams_by_batch.txt): >= 2400 tiles 2 groups (105 x L=200:
    2 groups 64.8 us/step, 3 66.5, 4 75.5; 70 replicas 46.0 / 47.0; cache-blocked 210
    and 420 replicas 131.9 / 256.5 us at 2 per wave vs 136.8 / 265.3 at 3), 1200-2400
    tiles 3 groups (35 replicas 27.4 vs 28.2 at 2, 52 replicas 36.2 vs 37.8), 300-1200
    tiles 2 groups (round 4, two agents per thread below 800 tiles: 8 x L=200 M=1 10.98 vs
    11.47 us/step, M=2 action 12.43 vs 13.89; 16 replicas 13.89 vs 15.78, 18.06 vs 20.90;
    profiles/r04/plan_sweep.txt), fewer tiles one group (4 replicas M=1 9.03 vs 9.36:
    cross-stream ordering costs more than it hides); never 4 at once
    (more streams than the 4 hardware queues serialise).  A batch whose state
    exceeds the Infinity-Cache budget is split into `waves` of groups that fit; the
    `resident` groups of a wave run concurrently and the next wave's groups queue
    behind them on the same streams.  `streams` overrides the group count; `single`
    (host-injected draws) forces one group."""
    if single:
        return 1, 1, 1
    waves = int(max(1, min(R, -(-(bytes_per_replica * R) // max(cache_bytes, 1)))))
    if streams is None:
        tw = min(L, 40)
        tiles = -(-L // tw) * -(-L // min(L, 25))
        tpw = R / waves * tiles
        per_wave = 2 if tpw >= 2400 else (3 if tpw >= 1200 else (2 if tpw >= 300 else 1))
        per_wave = int(max(1, min(per_wave, -(-R // waves))))
        streams = per_wave * waves if waves > 1 else per_wave
    groups = max(1, min(int(streams), R))
    resident = groups if waves == 1 else max(1, -(-groups // waves))
    return waves, groups, resident


# Library-made streams (spgg_stream_create) are pooled per library and device and outlive their
# engine: torch's pinned-memory allocator keeps the events of a pinned buffer's copies (run()'s
# stop flags) and queries them when it allocates again, so a stream destroyed under such an event
# made a later engine's pinned allocation fail (hipErrorCapturedEvent).  They are destroyed at
# interpreter exit, after a device sync and torch's pinned cache release, while the HIP runtime
# (and a profiler's interception of it) is still up.
_STREAM_POOL: dict = {}   # (library, device) -> free stream handles
_STREAM_OWNER: dict = {}  # every live pooled stream -> (library, device)


def _pool_key(lib, dev_index: int):
    return (getattr(lib, "_name", id(lib)), dev_index)


def _take_stream(lib, dev_index: int) -> int:
    free = _STREAM_POOL.setdefault(_pool_key(lib, dev_index), [])
    if free:
        return free.pop()
    h = ctypes.c_void_p()
    C.check(lib.spgg_stream_create(dev_index, ctypes.byref(h)), None, "spgg_stream_create")
    _STREAM_OWNER[h.value] = (lib, dev_index)
    return h.value


def _give_streams(handles) -> None:
    for h in handles:
        if h in _STREAM_OWNER:   # (not yet destroyed by the exit hook)
            lib, dev = _STREAM_OWNER[h]
            _STREAM_POOL.setdefault(_pool_key(lib, dev), []).append(h)


@atexit.register
def _destroy_streams() -> None:
    if not _STREAM_OWNER:
        return
    try:
        for dev in {d for _, d in _STREAM_OWNER.values()}:
            torch.cuda.synchronize(dev)
        torch._C._host_emptyCache()
    except Exception:
        pass
    for h, (lib, _) in list(_STREAM_OWNER.items()):
        lib.spgg_stream_destroy(h)
    _STREAM_OWNER.clear()
    _STREAM_POOL.clear()


class BatchEngine:
    """n_rep independent replicas of one (L, M, state) configuration on one device."""

    def __init__(self, L: int, iterations: int, replicas: Sequence[ReplicaParams],
                 use_second_order: bool = True, state_representation: str = "reputation",
                 rng: str = "mt19937", device=None, init: Optional[Sequence[InitState]] = None,
                 lib_path: Optional[str] = None, streams: Optional[int] = None,
                 algorithm: str = "qlearning", replica_offset: int = 0):
        if state_representation not in ("reputation", "action"):
            raise ValueError(f"Unknown state_representation: {state_representation}. "
                             f"Must be 'reputation' or 'action'")
        if rng not in C.RNG_MODES:
            raise ValueError(f"rng must be one of {sorted(C.RNG_MODES)}")
        if not torch.cuda.is_available():
            raise C.SpggError("BatchEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = C.load(lib_path)
        self.algorithm = canonical_name(algorithm)
        self.alg = C.ALGORITHMS[self.algorithm]
        self.double_q = self.alg == C.ALG_DOUBLE_Q
        self.QW = 8 if self.double_q else 4     # doubles per agent in the Q buffers
        self.L, self.n = int(L), int(L) * int(L)
        self.T = int(iterations)
        self.reps = list(replicas)
        self.R = len(self.reps)
        self.M2 = bool(use_second_order)
        self.state_rep = state_representation
        self.rng = rng
        # global index of replica 0 (a rank's shard offset): replica k's Philox stream id is
        # replica_offset + k, so its stream does not depend on how the sweep was sharded
        self.replica_offset = int(replica_offset)
        self.dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        if init is None:
            init = [reference_init(self.L, np.random.RandomState(p.seed), algorithm=self.algorithm)
                    for p in self.reps]
        self.init = list(init)
        if len(self.init) != self.R:
            raise ValueError("one InitState per replica")
        # Replica groups on separate HIP streams: their step kernels run
        # concurrently, so one group's tail / compute phase overlaps another
        # group's memory phase (a single launch moves in lockstep rounds).
        # Infinity-Cache blocking: a batch whose state exceeds the cache budget is
        # stepped in `waves` turns -- the groups of one wave run concurrently (one
        # stream each) for `chunk` iterations while the next wave's groups queue
        # behind them on the same streams (groups are independent: results are
        # unchanged, only the order of launches across groups)
        self.cache_bytes = int(float(tuning_env("SPGG_CACHE_MB", "240")) * 2**20)
        self.chunk = max(1, int(tuning_env("SPGG_CHUNK", "64")))
        self.enqueue_chunk = int(tuning_env("SPGG_ENQ_CHUNK", "8"))
        # resident replica groups enqueued iteration by iteration in one call (spgg_step_groups);
        # SPGG_INTERLEAVE=0: one spgg_step call per group and enqueue_chunk iterations
        self.interleave = tuning_env("SPGG_INTERLEAVE", "1") != "0"
        self.skip_dead = tuning_env("SPGG_SKIP_DEAD", "1") != "0"
        if streams is None and tuning_env("SPGG_STREAMS"):
            streams = int(tuning_env("SPGG_STREAMS")) or None
        self.waves, self.G, self.resident = plan_groups(
            self.R, self.L, self.state_bytes_per_replica(), self.cache_bytes, streams, single=rng == "inject")
        self._alloc()
        self._create()
        self.t = 1                 # next iteration to execute
        self.stopped = np.zeros(self.R, dtype=np.int64)
        self.snapshots = [dict() for _ in range(self.R)]
        self.png_frames = [dict() for _ in range(self.R)]
        self._flushed = False

    def state_bytes_per_replica(self) -> int:
        """Bytes of per-agent state one iteration reads and writes (Q, the S / R ping-pong,
        ~10 % border records; SARSA also the stored pending NI record md + atd, which the
        other operators' large-batch kernels recompute -- the batches this budget can split):
        the Infinity-Cache working set.  Budget SPGG_CACHE_MB
        (default 240 of the MI355X's 256 MB: measured knee for L=200 between 227 and 272 MB,
        profiles/r01/current/replicas_sweep_*)."""
        rsz = 1 if all(p.rep_unit() is not None for p in self.reps) else 8
        rec = 8 + 4 if self.alg == C.ALG_SARSA else 0
        return int(self.n * (self.QW * 8 + rec + 2 + 2 * rsz) * 1.1)

    # -- setup ---------------------------------------------------------------
    def _alloc(self):
        R, n, T, d = self.R, self.n, self.T, self.dev
        f64, u8 = torch.float64, torch.uint8
        S0 = np.stack([np.asarray(s.S).reshape(n) for s in self.init]).astype(np.uint8)
        if self.double_q:
            if any(s.tables is None for s in self.init):
                raise ValueError("double_qlearning needs both initial tables (InitState.tables)")
            Q0 = np.stack([to_state_planes(*s.tables) for s in self.init])
        else:
            Q0 = np.stack([to_state_planes(s.Q) for s in self.init])
        self.S = torch.zeros((2, R, n), dtype=u8, device=d)
        self.S[0].copy_(torch.from_numpy(S0))
        units = [p.rep_unit() for p in self.reps]
        self.rep_int8 = (all(u is not None for u in units)
                         and tuning_env("SPGG_REP_F64", "0") != "1")
        self.rep_units = np.array([u if u is not None else 1.0 for u in units])
        self.Rep = torch.zeros((2, R, n), dtype=torch.int8 if self.rep_int8 else f64, device=d)
        # Q updated in place, in state planes per replica (spgg_abi.h; to_state_planes)
        self.Qb = torch.from_numpy(np.ascontiguousarray(Q0)).to(d)
        # pending NI record, in place: max(0, max_diff) and |alpha*td'| (diagnostic)
        self.md = torch.zeros((R, n), dtype=f64, device=d)
        self.atd = torch.zeros((R, n), dtype=torch.float32, device=d)
        # draw records (device MT19937 / inject): a ring of bit planes, allocated in _create
        # from the library's layout (spgg_draw_layout)
        self.n_planes = C.DRAW_PLANES[self.alg]
        mt = np.zeros((R, 625), dtype=np.uint32)
        if self.rng == "mt19937":
            for k, s in enumerate(self.init):
                if s.mt_key is None:
                    raise ValueError("mt19937 mode needs the continuing MT19937 key of each replica")
                mt[k, :624] = s.mt_key
                mt[k, 624] = s.mt_pos
        self.mt_state = torch.from_numpy(mt.view(np.int32)).to(d)
        eps = np.zeros((R, T + 2))
        cache = {}
        for k, p in enumerate(self.reps):
            key = (p.epsilon, p.epsilon_decay, p.epsilon_min)
            if key not in cache:
                cache[key] = epsilon_table(*key, T + 1)
            eps[k] = cache[key]
        self.eps_host = eps
        self.eps = torch.from_numpy(eps).to(d)
        # history record [R][stripes][T+2][NSTAT]: allocated in _create (stripes per the library)
        self._ncoop0 = (S0 == 0).sum(axis=1).astype(np.float64)
        self.stop_iter = torch.zeros(R, dtype=torch.int32, device=d)
        self.P_buf = torch.zeros((R, n), dtype=f64, device=d)

    def _create(self):
        cfg = C.Config(device=self.dev.index, n_rep=self.R, L=self.L, second_order=int(self.M2),
                       state_mode=C.STATE_ACTION if self.state_rep == "action" else C.STATE_REPUTATION,
                       rng_mode=C.RNG_MODES[self.rng], iterations=self.T, rep_int8=int(self.rep_int8),
                       algorithm=self.alg, batch_reps=self.R)   # one tiling for every group
        params = [p.to_c() for p in self.reps]
        for k, p in enumerate(params):
            p.stream_id = self.replica_offset + k
        self.groups = []
        self._own_streams = []
        if self.G == 1:
            streams = [torch.cuda.current_stream(self.dev)]
        elif tuning_env("SPGG_OWN_STREAMS", "1") == "1":
            # streams made by the library (spgg_stream_create, SPGG_STREAM_MODE), not torch's pool:
            # torch's pool streams share HIP's few hardware queues with every earlier user, and
            # two streams on one queue run serialised (cfg3, a second engine in the process:
            # 80-82 us/iter on pool streams, 58.5-59 on the library's; profiles/r03/streams.txt)
            for _ in range(self.resident):
                self._own_streams.append(_take_stream(self.lib, self.dev.index))
            streams = [torch.cuda.ExternalStream(h, device=self.dev) for h in self._own_streams]
        else:
            streams = [torch.cuda.Stream(self.dev) for _ in range(self.resident)]
        bounds = np.linspace(0, self.R, self.G + 1).round().astype(int)
        for g in range(self.G):
            r0, r1 = int(bounds[g]), int(bounds[g + 1])
            cfg.n_rep = r1 - r0
            ctx = ctypes.c_void_p()
            C.check(self.lib.spgg_create(ctypes.byref(ctx), cfg), None, "spgg_create")
            self.groups.append(dict(r0=r0, r1=r1, ctx=ctx, stream=streams[g % len(streams)], live=True))
            arr = (C.RepParams * (r1 - r0))(*params[r0:r1])
            C.check(self.lib.spgg_set_params(ctx, arr), ctx, "spgg_set_params")
            # border records and history-record stripes: library-defined sizes, which the
            # shared buffers' per-replica strides assume to be the same for every group
            layout = self._layout(ctx) + (self._draw_layout(ctx), self._mt_chains(ctx))
            if g == 0:
                self.layout = layout
                tile, per, self.stripes = layout[:3]
                self.pub = torch.zeros((2, self.R, max(1, per)), dtype=torch.float64, device=self.dev)
                self.stats = torch.zeros((self.R, self.stripes, self.T + 2, C.NSTAT), dtype=torch.float64,
                                         device=self.dev)
                self.stats[:, 0, 1, C.ST_NCOOP] = torch.from_numpy(self._ncoop0).to(self.dev)
                slots, words, snaps = self._draw_layout(ctx)
                self.draw_slots, self.draw_words = slots, words
                rngd = self.rng != "philox"
                self.draws = torch.zeros((slots, self.R, words) if rngd else (1, 1, 1), dtype=torch.int32,
                                         device=self.dev)
                self.mt_snap = torch.zeros((snaps, self.R, 625) if self.rng == "mt19937" else (1, 1, 1),
                                           dtype=torch.int32, device=self.dev)
            elif layout != self.layout:
                raise C.SpggError(f"replica group {g} got layout {layout} != group 0's {self.layout} "
                                  "(tile, border-record doubles, stripes, draw ring, MT chains): shared buffer "
                                  "strides would disagree")
            b = C.Buffers()   # the group's replica slice of every buffer
            for i in range(2):
                b.S[i], b.R[i] = self.S[i][r0].data_ptr(), self.Rep[i][r0].data_ptr()
                b.pub[i] = self.pub[i][r0].data_ptr()
            b.Q, b.md, b.atd = self.Qb[r0].data_ptr(), self.md[r0].data_ptr(), self.atd[r0].data_ptr()
            b.draws = self.draws[0, min(r0, self.draws.shape[1] - 1)].data_ptr()
            b.draw_slot_stride = self.draws.shape[1] * self.draws.shape[2]
            b.mt_state = self.mt_state[r0].data_ptr()
            b.mt_snap = self.mt_snap[0, min(r0, self.mt_snap.shape[1] - 1)].data_ptr()
            b.mt_snap_stride = self.mt_snap.shape[1] * self.mt_snap.shape[2]
            b.eps, b.stats = self.eps[r0].data_ptr(), self.stats[r0].data_ptr()
            b.stop_iter = self.stop_iter[r0].data_ptr()
            C.check(self.lib.spgg_bind(ctx, b), ctx, "spgg_bind")
            self.groups[-1]["bufs"] = b
        self.streams = streams
        self._draw_stream = None
        if self.rng == "mt19937" and self.G > 1 and tuning_env("SPGG_SHARED_DRAW_STREAM", "1") == "1":
            # one generator stream for every group (spgg_set_draw_stream) instead of one per context:
            # the groups' generator chunks run one after the other instead of side by side, so half
            # as many generator workgroups share the CUs with the step launches at any time (cfg3
            # whole run 68.0 -> 65.9 us/iter, profiles/r06/mt_generator/).  A torch pool stream:
            # non-blocking, and never on the hardware queue of a CU-masked group stream.
            self._draw_stream = torch.cuda.Stream(self.dev)
            for gr in self.groups:
                C.check(self.lib.spgg_set_draw_stream(gr["ctx"], ctypes.c_void_p(self._draw_stream.cuda_stream)),
                        gr["ctx"], "spgg_set_draw_stream")
        self.ctx = self.groups[0]["ctx"]
        self.tile = self.layout[0]
        self.mt_layout = self.layout[4]
        # persistent launches (spgg_persistent): every tile of the batch fits the device at once, so
        # each step call (MT19937: each generator chunk of it) is one launch per group
        on, cap = ctypes.c_int32(), ctypes.c_int32()
        C.check(self.lib.spgg_persistent(self.ctx, ctypes.byref(on), ctypes.byref(cap)), self.ctx, "spgg_persistent")
        self.persistent, self.persist_capacity = bool(on.value), int(cap.value)

    def _draw_layout(self, ctx):
        """(ring slots, u32 words per replica and slot, key-snapshot slots) of the draw records."""
        slots, snaps, words = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        C.check(self.lib.spgg_draw_layout(ctx, ctypes.byref(slots), ctypes.byref(words), ctypes.byref(snaps)),
                ctx, "spgg_draw_layout")
        return int(slots.value), int(words.value), int(snaps.value)

    def _mt_chains(self, ctx):
        """(chains per replica, iterations per chain) of the MT19937 generator (1, 1 otherwise)."""
        ch, per = ctypes.c_int32(), ctypes.c_int32()
        C.check(self.lib.spgg_mt_chains(ctx, ctypes.byref(ch), ctypes.byref(per)), ctx, "spgg_mt_chains")
        return int(ch.value), int(per.value)

    def check_status(self):
        """Raise if a replica group's draw generator reported an error (spgg_status: the pinned
        copy of its error word after the last completed chunk; no sync)."""
        for g in self.groups:
            f = ctypes.c_uint32()
            C.check(self.lib.spgg_status(g["ctx"], ctypes.byref(f)), g["ctx"], "spgg_status")
            if f.value:
                raise C.SpggError(f"replica group {self.groups.index(g)}: the MT19937 draw generator failed "
                                  f"(error word {f.value}); the run's draws are not the reference's")

    def draw_record(self, t):
        """(planes, R, n) uint8 0/1 view of iteration t's draw record (unpacked on the host)."""
        x = self.draws[(t - 1) % self.draw_slots].cpu().numpy().view(np.uint32)
        x = x.reshape(self.R, -1, self.n_planes).transpose(0, 2, 1)          # [R][planes][words]
        bits = np.unpackbits(np.ascontiguousarray(x).view(np.uint8), axis=-1, bitorder="little")
        return np.ascontiguousarray(bits[..., :self.n].transpose(1, 0, 2))

    def _layout(self, ctx):
        """(tile shape, border-record doubles per replica, history stripes) of a context."""
        tw, th = ctypes.c_int32(), ctypes.c_int32()
        C.check(self.lib.spgg_tile_shape(ctx, ctypes.byref(tw), ctypes.byref(th)), ctx, "spgg_tile_shape")
        per = ctypes.c_int64()
        C.check(self.lib.spgg_pub_doubles(ctx, ctypes.byref(per)), ctx, "spgg_pub_doubles")
        ns = ctypes.c_int32()
        C.check(self.lib.spgg_stat_stripes(ctx, ctypes.byref(ns)), ctx, "spgg_stat_stripes")
        return (tw.value, th.value), int(per.value), int(ns.value)

    def _enqueue(self, fn, rounds=(None,)):
        """For each round, run fn(group, stream_handle[, round]) on every group's
        stream, all ordered after the current stream's prior work and before its
        later work.  Groups sharing a stream (cache blocking) run in turn."""
        cur = torch.cuda.current_stream(self.dev)
        call = (lambda g, s, r: fn(g, s)) if rounds == (None,) else fn
        if self.G == 1:
            for r in rounds:
                call(self.groups[0], cur.cuda_stream, r)
            return
        for st in self.streams:
            st.wait_stream(cur)
        for r in rounds:
            for g in self.groups:
                call(g, g["stream"].cuda_stream, r)
        for st in self.streams:
            cur.wait_stream(st)

    def close(self):
        for g in getattr(self, "groups", []):
            if g.get("ctx"):
                self.lib.spgg_destroy(g["ctx"])
                g["ctx"] = None
        self.groups = []
        self.ctx = None
        if getattr(self, "_own_streams", None):
            torch.cuda.synchronize(self.dev)
            self.streams = []
            _give_streams(self._own_streams)
            self._own_streams = []
            self._loop = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    # -- stepping ------------------------------------------------------------
    def _inject(self, t):
        """Host draws of iteration t, in the reference's order, for replicas that
        execute it: every select draws rand then randint (algorithms.py:105,108);
        SARSA selects three times (spgg.py:410,434,452); Double-Q then draws its
        table choice (algorithms.py:302)."""
        ncoop = self.stats[:, :, t, C.ST_NCOOP].sum(dim=1).cpu().numpy()
        stop = self.stop_iter.cpu().numpy()
        planes = np.zeros((self.n_planes, self.R, self.n), dtype=np.uint8)
        L = self.L
        for k, s in enumerate(self.init):
            if stop[k] != 0 or ncoop[k] == 0 or ncoop[k] == self.n:
                continue
            e = self.eps_host[k, t]
            selects = 3 if self.alg == C.ALG_SARSA else 1
            for j in range(selects):
                planes[2 * j, k] = s.rs.rand(L, L).reshape(-1) < e
                planes[2 * j + 1, k] = s.rs.randint(0, 2, size=(L, L)).reshape(-1)
            if self.double_q:
                planes[2, k] = s.rs.rand(L, L).reshape(-1) < 0.5
        # bits, 32 agents per word, the planes of a word interleaved (spgg_abi.h draws)
        nwords = self.draw_words // self.n_planes
        pad = np.zeros((self.n_planes, self.R, nwords * 32), dtype=np.uint8)
        pad[:, :, :self.n] = planes
        words = np.packbits(pad, axis=-1, bitorder="little").view(np.uint32)    # [planes][R][words]
        rec = np.ascontiguousarray(words.transpose(1, 2, 0)).reshape(self.R, -1)
        self.draws[(t - 1) % self.draw_slots].copy_(torch.from_numpy(rec.view(np.int32)))

    def launch_streams(self):
        """The torch streams this engine's step launches run on: the replica groups' streams, or
        the current stream for a single group (for events recorded beside the launches)."""
        if self.G == 1:
            return [torch.cuda.current_stream(self.dev)]
        return list(self.streams)

    def step(self, n_steps: int, ordered: bool = True):
        """Enqueue the next n_steps iterations (no host sync except in inject mode).

        ordered=False (every group resident): the groups' streams are NOT ordered after the
        current stream's earlier work nor it after theirs -- for a caller that has synchronised
        the device before and synchronises it after (bench.py's timed window).  Each of those two
        cross-stream waits costs a window ~60 us of latency on MI355X / ROCm 7 (cfg3, 20
        iterations: 63.4 -> 57.1 us/step without both; tools/window_timeline.py)."""
        n_steps = min(n_steps, self.T - self.t + 1)
        if n_steps <= 0:
            return 0
        if self.rng == "inject":
            for _ in range(n_steps):
                self._inject(self.t)
                C.check(self.lib.spgg_step(self.ctx, self.t, 1, self.stream), self.ctx, "spgg_step")
                self.t += 1
        else:
            t0, end = self.t, self.t + n_steps
            live = [g for g in self.groups if g["live"]]
            if self.G > 1 and self.resident == self.G and self.interleave and live:
                # every group resident: one call enqueues all of them iteration by iteration
                # (spgg_step_groups), so every group's stream starts within one launch of the
                # first instead of one host call of k launches per group later (cfg3, 20
                # iterations after 400: 60.0 -> 57.8 us/step for k = 8 -> 1)
                key = tuple(id(g) for g in live)   # the call's arrays, made once per live set
                if getattr(self, "_groups_args", (None,))[0] != key:
                    self._groups_args = (key, (ctypes.c_void_p * len(live))(*[g["ctx"] for g in live]),
                                         (ctypes.c_void_p * len(live))(*[g["stream"].cuda_stream for g in live]))
                _, ctxs, strs = self._groups_args
                cur = torch.cuda.current_stream(self.dev)  # ordered as _enqueue orders its rounds
                if ordered:
                    for st in self.streams:
                        st.wait_stream(cur)
                C.check(self.lib.spgg_step_groups(ctxs, strs, len(live), t0, n_steps), live[0]["ctx"],
                        "spgg_step_groups")
                if ordered:
                    for st in self.streams:
                        cur.wait_stream(st)
                self.t += n_steps
                return n_steps
            # groups are enqueued round-robin, k iterations at a time: with every group
            # resident this only interleaves the host's launches across the streams (all
            # of them start within k launches, instead of the last group waiting for the
            # host to enqueue every other group's n_steps); with cache blocking it is
            # also the turn length of a wave
            k = self.chunk if self.resident < self.G else self.enqueue_chunk
            chunks = [(t, min(k, end - t)) for t in range(t0, end, k)] if k > 0 else [(t0, n_steps)]
            self._enqueue(lambda g, s, c: g["live"] and C.check(self.lib.spgg_step(g["ctx"], c[0], c[1], s),
                                                                g["ctx"], "spgg_step"), rounds=chunks)
            self.t += n_steps
        return n_steps

    def all_stopped(self) -> bool:
        """Host check of the absorbing stops (a sync of the current stream); retires groups
        whose replicas have all stopped (_note_stops)."""
        return self._note_stops(self.stop_iter.cpu().numpy())

    def flush(self):
        """Apply the deferred NI term of the last executed iteration (once, at the end)."""
        if self._flushed or self.t <= 1:
            return
        tl = self.t - 1
        self._enqueue(lambda g, s: C.check(self.lib.spgg_flush(g["ctx"], tl, s), g["ctx"], "spgg_flush"))
        self._flushed = True

    def _note_stops(self, stop) -> bool:
        """Absorbing stops as of some enqueued iteration: retire groups whose replicas have all
        stopped (their later launches would only stage loads and exit), raise on a generator
        error; True once every replica has stopped."""
        self.stopped = np.asarray(stop).astype(np.int64)
        self.check_status()
        if self.skip_dead:
            for g in self.groups:
                if g["live"] and np.all(self.stopped[g["r0"]:g["r1"]] != 0):
                    g["live"] = False
        return bool(np.all(self.stopped != 0))

    def _loop_stream(self):
        """The stream run() orders its turns, stop-flag copies and host syncs on, instead of the
        legacy null stream -- which every blocking stream (the CU-masked group and MT19937
        generator streams) synchronises with, so a host sync there drained the generator's
        queued chunks at every turn.  Replica groups: group 0's stream (a fifth stream would
        share one of the 4 hardware queues: cfg3 MT19937 whole run 92.6 us/iter on a stream of
        its own, 78.7 on the null stream, 71.9 on group 0's); one group: a library-made
        stream (cfg5 MT19937 whole run 27.4 vs 32.3 on the null stream, cfg2 10.0 vs 11.1).
        profiles/r04/turns_and_loop_stream.txt."""
        if self.G > 1:
            return self.streams[0]
        if getattr(self, "_loop", None) is None:
            h = _take_stream(self.lib, self.dev.index)
            self._own_streams.append(h)
            self._loop = torch.cuda.ExternalStream(h, device=self.dev)
        return self._loop

    def run(self, chunk: int = 256, snapshots: bool = True, png: bool = False,
            progress: Optional[Callable[[int], None]] = None):
        """Execute iterations until `iterations` or every replica is absorbed.

        Turns of `chunk` iterations.  The absorbing-stop check of a turn is an asynchronous
        copy of the stop flags; the host reads it one turn later, so the device never idles
        at a turn boundary.  The price of the lag: once every replica has absorbed, one more
        turn is already enqueued (up to `chunk` step launches that return after their loads,
        plus MT19937 generator chunks), and a group is retired one turn late.  Absorbed
        replicas' launches change nothing, so results are unaffected; only the wall time of a
        run that absorbs early carries that turn.  Snapshot iterations sync."""
        stops = set()
        if snapshots:
            stops |= {i for i in SNAPSHOT_ITERS if i <= self.T}
        if png:
            stops |= {i + 1 for i in PNG_ITERS if i + 1 <= self.T + 1}
        caller = torch.cuda.current_stream(self.dev)
        loop = self._loop_stream()
        loop.wait_stream(caller)
        flags = torch.empty((2, self.R), dtype=torch.int32, pin_memory=True)
        pending = []   # (event, slot) of the stop-flag copies in flight (<= 2: this turn's, the last one's)
        turn = 0
        done = False
        with torch.cuda.stream(loop):
            while self.t <= self.T and not done:
                if self.t in stops:
                    self._capture(self.t, snapshots and self.t in SNAPSHOT_ITERS,
                                  png and (self.t - 1) in PNG_ITERS)
                    pending = []   # (_capture synchronised the stream)
                    done = self._note_stops(self.stop_iter.cpu().numpy())
                    if done:
                        break
                nxt = min([s for s in stops if s > self.t] + [self.t + chunk, self.T + 1])
                self.step(nxt - self.t)
                if progress:
                    progress(self.t - 1)
                slot, turn = turn & 1, turn + 1
                flags[slot].copy_(self.stop_iter, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(loop)
                pending.append((ev, slot))
                if len(pending) == 2:   # the previous turn's flags (this turn is still running)
                    ev0, s0 = pending.pop(0)
                    ev0.synchronize()
                    done = self._note_stops(flags[s0].numpy())
            if png and self.t in stops and (self.t - 1) in PNG_ITERS:
                self._capture(self.t, False, True)
            self.flush()
        caller.wait_stream(loop)
        torch.cuda.synchronize(self.dev)
        self._note_stops(self.stop_iter.cpu().numpy())

    def _capture(self, t, snap, png):
        """Host copies of S_t / R_t at iteration start (spgg.py:397-402) and of the
        strategies after iteration t-1 for the PNG snapshot (spgg.py:553-559)."""
        stop = self.stop_iter.cpu().numpy()
        cur = (t - 1) & 1
        S = self.S[cur].cpu().numpy() & 1
        Rn = self._rep_host(cur) if snap else None
        for k in range(self.R):
            if stop[k] != 0:
                continue
            if snap:
                self.snapshots[k][t] = (Rn[k].reshape(self.L, self.L).copy(),
                                        S[k].reshape(self.L, self.L).astype(np.int64))
            if png:
                self.png_frames[k][t - 1] = S[k].reshape(self.L, self.L).astype(np.int64)

    # -- results -------------------------------------------------------------
    def last_iteration(self, k) -> int:
        """Iterations with a start record (incl. the absorbing one)."""
        s = int(self.stopped[k])
        return s if s else self.t - 1

    def final_state(self, k):
        """(Q (L,L,2,2), R (L,L), S (L,L) int64) of replica k after the run."""
        last = self.last_iteration(k)
        s = int(self.stopped[k])
        if s:   # absorbed at s: S_s, R_s untouched since; Q finalized by launch s
            cur = (s - 1) & 1
        else:   # S_{last+1}, R_{last+1}; Q finalized by the flush launch last+1
            cur = last & 1
        L = self.L
        tabs = from_state_planes(self.Qb[k].cpu().numpy(), L, self.double_q)
        if self.double_q:   # q_table = mean of the two tables (algorithms.py:262-266)
            Q = (tabs[0] + tabs[1]) / 2
        else:
            Q = tabs[0]
        R = self._rep_host(cur)[k].reshape(L, L)
        S = (self.S[cur, k].cpu().numpy() & 1).reshape(L, L).astype(np.int64)
        return Q, R, S

    def final_tables(self, k):
        """Double-Q: (q_table_1, q_table_2) of replica k after the run."""
        if not self.double_q:
            raise ValueError("final_tables: not a double_qlearning engine")
        return from_state_planes(self.Qb[k].cpu().numpy(), self.L, True)

    def _rep_host(self, buf):
        """R plane `buf` of every replica as float64 (exact k*unit in compact mode)."""
        x = self.Rep[buf].cpu().numpy()
        if self.rep_int8:
            return x.astype(np.float64) * self.rep_units[:, None]
        return x

    def payoff_at(self, t):
        """P from S_t for every replica (device kernel), as (R, L, L) float64."""
        self._enqueue(lambda g, s: C.check(
            self.lib.spgg_payoff(g["ctx"], int(t), self.P_buf[g["r0"]].data_ptr(), s), g["ctx"], "spgg_payoff"))
        return self.P_buf.cpu().numpy().reshape(self.R, self.L, self.L)

    def finalize_history(self):
        """Derived history slots (payoff sums, w_P*P, w_rep*rr, reward over D) of every
        executed iteration from the counted ones (spgg_history_finalize; idempotent)."""
        tl = self.t - 1
        if tl >= 1:
            self._enqueue(lambda g, s: C.check(self.lib.spgg_history_finalize(g["ctx"], tl, s), g["ctx"],
                                               "spgg_history_finalize"))

    def stats_folded(self):
        """(R, T+2, NSTAT) device tensor of the history record: stripes summed, GMAX maxed."""
        self.finalize_history()
        st = self.stats.sum(dim=1)
        if self.stripes > 1:
            st[..., C.ST_GMAX] = self.stats[..., C.ST_GMAX].amax(dim=1)
        return st

    def mt_state_host(self, k):
        st = self.mt_state[k].cpu().numpy().view(np.uint32)
        return st[:624].copy(), int(st[624])

    def histories(self):
        """Per-replica dict of the reference's per-iteration datasets (spgg.py:595-618)."""
        st = self.stats_folded().cpu().numpy()
        return [histories_from_stats(st[k], self.last_iteration(k), int(self.stopped[k]) != 0,
                                     self.eps_host[k], self.n) for k in range(self.R)]

    def gmax_history(self, k):
        st = self.stats_folded()[k, :, C.ST_GMAX].cpu().numpy()
        last = self.last_iteration(k)
        m = last - 1 if int(self.stopped[k]) else last
        return st[1:m + 1]


_STEP_KEYS = (
    ["switch_C_to_D", "switch_D_to_C", "neighbor_influence_percent",
     "payoff_component_history", "rep_component_history",
     "best_neighbor_second_order_percent", "reputation_reward_ratio",
     "avg_reward_C_history", "avg_reward_D_history"]
    + [f"group_comp_d{d}_history" for d in range(6)]
    + [f"{g}_q_{s}_{a}_history" for g in ("cooperators", "defectors")
       for s in ("s0", "s1") for a in ("c", "d")]
    + [f"avg_q_{s}_{a}_history" for s in ("s0", "s1") for a in ("c", "d")]
)


def histories_from_stats(S, last, stopped, eps_row, n):
    """Turn one replica's device history record into the reference's datasets.

    S: (iterations+2, NSTAT) float64 record; last: iterations with a start
    record (incl. an absorbing one); stopped: absorbed at `last`; eps_row: eps
    table (eps_row[t] = eps used by iteration t).  Means are sum/count, as
    np.mean (spgg.py:383-394, 419-426, 511-592); empty masks give the
    reference's 0 / NaN.
    """
    n = float(n)
    m = last - 1 if stopped else last
    it = S[1:last + 1]
    nc = it[:, C.ST_NCOOP]
    nd = n - nc
    ds = {}
    ds["coop_rate_history"] = nc / n
    sump = it[:, C.ST_SUMP]
    ds["it_records_final"] = np.stack([
        nc / n, nd / n, sump, sump / n,
        np.where(nc > 0, it[:, C.ST_SUMP_C] / np.maximum(nc, 1), 0.0),
        np.where(nd > 0, it[:, C.ST_SUMP_D] / np.maximum(nd, 1), 0.0)], axis=1).reshape(-1, 6)
    ds["rep_avg_history_final"] = it[:, C.ST_SUMR] / n
    if m == 0:
        empty = np.array([])
        for key in _STEP_KEYS:
            ds[key] = empty
        ds["epsilon_history_final"] = empty
        return ds
    st_m = S[1:m + 1]
    nc_m = st_m[:, C.ST_NCOOP]            # prev_S == 0 count of step i
    nc_d = n - nc_m
    na_c = S[2:m + 2, C.ST_NCOOP]         # a == 0 count of step i
    na_d = n - na_c
    ds["epsilon_history_final"] = np.array(eps_row[2:m + 2], dtype=np.float64)
    ds["switch_C_to_D"] = st_m[:, C.ST_SW_CD].astype(np.int64)
    ds["switch_D_to_C"] = st_m[:, C.ST_SW_DC].astype(np.int64)
    ds["neighbor_influence_percent"] = st_m[:, C.ST_SUM_PCT] / n
    ds["payoff_component_history"] = st_m[:, C.ST_SUM_WPP] / n
    ds["rep_component_history"] = st_m[:, C.ST_SUM_WRR] / n
    npos = st_m[:, C.ST_NMD_POS]
    ds["best_neighbor_second_order_percent"] = np.where(
        npos > 0, st_m[:, C.ST_NMD_POS2] / np.maximum(npos, 1) * 100, 0.0)
    ds["reputation_reward_ratio"] = np.where(
        na_c > 0, st_m[:, C.ST_SUM_RATIO_C] / np.maximum(na_c, 1), np.nan)
    ds["avg_reward_C_history"] = np.where(na_c > 0, st_m[:, C.ST_SUM_REW_C] / np.maximum(na_c, 1), 0.0)
    ds["avg_reward_D_history"] = np.where(na_d > 0, st_m[:, C.ST_SUM_REW_D] / np.maximum(na_d, 1), 0.0)
    for d in range(6):
        ds[f"group_comp_d{d}_history"] = (st_m[:, C.ST_GC0 + d] / n) * 100
    for s_i, s_n in enumerate(("s0", "s1")):
        for a_i, a_n in enumerate(("c", "d")):
            e = 2 * s_i + a_i
            ds[f"cooperators_q_{s_n}_{a_n}_history"] = np.where(
                nc_m > 0, st_m[:, C.ST_SUMQ_C + e] / np.maximum(nc_m, 1), np.nan)
            ds[f"defectors_q_{s_n}_{a_n}_history"] = np.where(
                nc_d > 0, st_m[:, C.ST_SUMQ_D + e] / np.maximum(nc_d, 1), np.nan)
            ds[f"avg_q_{s_n}_{a_n}_history"] = st_m[:, C.ST_SUMQ + e] / n
    return ds
