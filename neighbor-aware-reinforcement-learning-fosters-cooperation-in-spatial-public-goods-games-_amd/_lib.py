"""ctypes binding of libspgg_hip.so (C ABI declared in include/spgg_abi.h).

The library is built in-tree by `build.py` (hipcc --offload-arch=gfx950).  There
is no fallback: if the shared object is missing or cannot be loaded, every entry
point raises, so a GPU run can never silently take another path.
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libspgg_hip.so")

ABI_VERSION = 16
OK, E_ARG, E_STATE, E_HIP = 0, -1, -2, -3
GEN_ERR_SPIN = 1
STATE_REPUTATION, STATE_ACTION = 0, 1
RNG_INJECT, RNG_MT19937, RNG_PHILOX = 0, 1, 2
RNG_MODES = {"inject": RNG_INJECT, "mt19937": RNG_MT19937, "philox": RNG_PHILOX}
ALG_QLEARNING, ALG_SARSA, ALG_EXPECTED_SARSA, ALG_DOUBLE_Q = 0, 1, 2, 3
ALGORITHMS = {"qlearning": ALG_QLEARNING, "sarsa": ALG_SARSA, "expected_sarsa": ALG_EXPECTED_SARSA,
              "double_qlearning": ALG_DOUBLE_Q}
DRAW_PLANES = {ALG_QLEARNING: 2, ALG_SARSA: 6, ALG_EXPECTED_SARSA: 2, ALG_DOUBLE_Q: 3}

# stats record layout (enum in spgg_abi.h)
ST_NCOOP, ST_SUMP, ST_SUMP_C, ST_SUMP_D, ST_SUMR = 0, 1, 2, 3, 4
ST_SW_CD, ST_SW_DC, ST_SUM_WPP, ST_SUM_WRR = 5, 6, 7, 8
ST_SUM_REW_C, ST_SUM_REW_D, ST_SUM_RATIO_C = 9, 10, 11
ST_GC0, ST_NMD_POS, ST_NMD_POS2, ST_SUM_PCT = 12, 18, 19, 20
ST_SUMQ, ST_SUMQ_C, ST_SUMQ_D, ST_GMAX = 21, 25, 29, 33
NSTAT = 34

EXPORTED = ("spgg_abi_version", "spgg_build_id", "spgg_last_error", "spgg_create", "spgg_set_params",
            "spgg_bind", "spgg_step", "spgg_step_groups", "spgg_flush", "spgg_draw", "spgg_payoff", "spgg_tile_shape",
            "spgg_destroy", "spgg_draw_planes", "spgg_pub_doubles", "spgg_stat_stripes",
            "spgg_history_finalize", "spgg_draw_layout", "spgg_set_draw_stream", "spgg_draw_range",
            "spgg_mt_chains", "spgg_mt_jump_poly", "spgg_stream_create", "spgg_stream_destroy",
            "spgg_status", "spgg_persistent")
# test-only entry points (include/spgg_test.h): exported by the library, not part of the product ABI
TEST_EXPORTED = ("spgg_test_set_error",)


class Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("n_rep", ctypes.c_int32), ("L", ctypes.c_int32),
                ("second_order", ctypes.c_int32), ("state_mode", ctypes.c_int32),
                ("rng_mode", ctypes.c_int32), ("iterations", ctypes.c_int32),
                ("rep_int8", ctypes.c_int32), ("algorithm", ctypes.c_int32),
                ("batch_reps", ctypes.c_int32)]


class RepParams(ctypes.Structure):
    _fields_ = [(name, ctypes.c_double) for name in (
        "rc", "cost", "norm_min", "norm_den", "w_p", "w_rep", "alpha", "gamma",
        "diag_alpha", "diag_gamma", "kappa", "lambda_eps", "rep_gain_c", "neg_delta_r_d",
        "r_min", "r_max")] + [("seed", ctypes.c_uint64), ("stream_id", ctypes.c_uint64),
                              ("pay_c", ctypes.c_double * 6), ("pay_d", ctypes.c_double * 6),
                              ("rep_unit", ctypes.c_double), ("rk_gain", ctypes.c_int32),
                              ("rk_loss", ctypes.c_int32), ("rk_min", ctypes.c_int32),
                              ("rk_max", ctypes.c_int32), ("norm_rcp", ctypes.c_double)]


class Buffers(ctypes.Structure):
    _fields_ = [("S", ctypes.c_void_p * 2), ("R", ctypes.c_void_p * 2), ("Q", ctypes.c_void_p),
                ("pub", ctypes.c_void_p * 2), ("md", ctypes.c_void_p), ("atd", ctypes.c_void_p),
                ("draws", ctypes.c_void_p), ("draw_slot_stride", ctypes.c_int64),
                ("mt_state", ctypes.c_void_p), ("mt_snap", ctypes.c_void_p), ("mt_snap_stride", ctypes.c_int64),
                ("eps", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("stop_iter", ctypes.c_void_p)]


class SpggError(RuntimeError):
    pass


_libs = {}
_lock = threading.Lock()


def load(path: str | None = None):
    """Load (once per path) and type the shared library; raises if it is absent.

    `path` / $SPGG_LIB select a tuning build (A/B timing); each path gets its
    own RTLD_LOCAL handle, so variants can coexist in one process."""
    with _lock:
        p = path or os.environ.get("SPGG_LIB") or LIB_PATH
        if p in _libs:
            return _libs[p]
        if not os.path.exists(p):
            raise SpggError(f"{p} is not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(p)
        vp, i32 = ctypes.c_void_p, ctypes.c_int32
        lib.spgg_abi_version.restype = ctypes.c_int
        lib.spgg_abi_version.argtypes = []
        lib.spgg_last_error.restype = ctypes.c_char_p
        lib.spgg_last_error.argtypes = [vp]
        lib.spgg_create.restype = ctypes.c_int
        lib.spgg_create.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(Config)]
        lib.spgg_set_params.restype = ctypes.c_int
        lib.spgg_set_params.argtypes = [vp, ctypes.POINTER(RepParams)]
        lib.spgg_bind.restype = ctypes.c_int
        lib.spgg_bind.argtypes = [vp, ctypes.POINTER(Buffers)]
        lib.spgg_step.restype = ctypes.c_int
        lib.spgg_step.argtypes = [vp, i32, i32, vp]
        lib.spgg_step_groups.restype = ctypes.c_int
        lib.spgg_step_groups.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), i32, i32, i32]
        lib.spgg_flush.restype = ctypes.c_int
        lib.spgg_flush.argtypes = [vp, i32, vp]
        lib.spgg_history_finalize.restype = ctypes.c_int
        lib.spgg_history_finalize.argtypes = [vp, i32, vp]
        lib.spgg_draw.restype = ctypes.c_int
        lib.spgg_draw.argtypes = [vp, i32, vp]
        lib.spgg_draw_range.restype = ctypes.c_int
        lib.spgg_draw_range.argtypes = [vp, i32, i32, vp]
        lib.spgg_payoff.restype = ctypes.c_int
        lib.spgg_payoff.argtypes = [vp, i32, vp, vp]
        lib.spgg_tile_shape.restype = ctypes.c_int
        lib.spgg_tile_shape.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        lib.spgg_persistent.restype = ctypes.c_int
        lib.spgg_persistent.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        lib.spgg_destroy.restype = ctypes.c_int
        lib.spgg_destroy.argtypes = [vp]
        lib.spgg_draw_planes.restype = ctypes.c_int
        lib.spgg_draw_planes.argtypes = [i32]
        lib.spgg_stat_stripes.restype = ctypes.c_int
        lib.spgg_stat_stripes.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
        lib.spgg_pub_doubles.restype = ctypes.c_int
        lib.spgg_pub_doubles.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
        lib.spgg_draw_layout.restype = ctypes.c_int
        lib.spgg_draw_layout.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(i32)]
        lib.spgg_mt_chains.restype = ctypes.c_int
        lib.spgg_mt_chains.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        lib.spgg_mt_jump_poly.restype = ctypes.c_int
        lib.spgg_mt_jump_poly.argtypes = [ctypes.c_int64, vp]
        lib.spgg_stream_create.restype = ctypes.c_int
        lib.spgg_stream_create.argtypes = [i32, ctypes.POINTER(vp)]
        lib.spgg_stream_destroy.restype = ctypes.c_int
        lib.spgg_stream_destroy.argtypes = [vp]
        lib.spgg_set_draw_stream.restype = ctypes.c_int
        lib.spgg_set_draw_stream.argtypes = [vp, vp]
        lib.spgg_status.restype = ctypes.c_int
        lib.spgg_status.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32)]
        lib.spgg_test_set_error.restype = ctypes.c_int
        lib.spgg_test_set_error.argtypes = [vp, ctypes.c_uint32]
        lib.spgg_build_id.restype = ctypes.c_char_p
        lib.spgg_build_id.argtypes = []
        v = lib.spgg_abi_version()
        if v != ABI_VERSION:
            raise SpggError(f"libspgg_hip ABI {v} != expected {ABI_VERSION}")
        if p == LIB_PATH:   # the in-tree library must be built from these sources (a tuning
            from . import build as B   # build named by path / $SPGG_LIB is the caller's choice)
            if os.path.exists(B.SRC[0]):
                want, have = B.build_id(), lib.spgg_build_id().decode()
                if want != have:
                    raise SpggError(f"{p} was built from other sources (build id {have}, sources {want}); "
                                    "rebuild: python -c 'import __graft_entry__ as g; g.build()'")
        _libs[p] = lib
        return lib


def check(rc: int, ctx=None, what: str = "", lib=None):
    if rc != OK:
        lib = lib or load()
        detail = (lib.spgg_last_error(ctx) or b"").decode()  # ctx None: last spgg_create failure
        raise SpggError(f"{what} failed (rc={rc}): {detail}")
