"""The C-ABI library (CPU-side checks only, no device calls): it loads, reports the
header's ABI version, and exports every function include/spgg_abi.h declares -- the
set the ctypes binding types (spgg_amd/_lib.py EXPORTED)."""
import ctypes
import os
import re

import pytest

from spgg_amd import _lib

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADER = os.path.join(INCLUDE, "spgg_abi.h")
TEST_HEADER = os.path.join(INCLUDE, "spgg_test.h")


def _declared(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(spgg_\w+)\s*\(", src, flags=re.M))


def test_header_declares_the_bound_functions():
    """The product header declares exactly the product binding; the test hooks live in
    spgg_test.h alone (never in the product ABI a reference-side binding copies)."""
    assert _declared() == set(_lib.EXPORTED)
    assert _declared(TEST_HEADER) == set(_lib.TEST_EXPORTED)
    assert not set(_lib.TEST_EXPORTED) & _declared()


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [name for name in sorted(_declared() | _declared(TEST_HEADER)) if not hasattr(lib, name)]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_abi_version_matches_header():
    v = int(re.search(r"#define SPGG_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    lib = _lib.load()
    assert lib.spgg_abi_version() == v == _lib.ABI_VERSION


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_argument_errors_without_device():
    """Null arguments fail with SPGG_E_ARG before any device call."""
    lib = _lib.load()
    assert lib.spgg_create(None, None) == _lib.E_ARG
    assert lib.spgg_step(None, 1, 1, None) == _lib.E_ARG
    assert lib.spgg_draw_planes(7) == _lib.E_ARG
    assert lib.spgg_draw_planes(_lib.ALG_SARSA) == 6
    n = ctypes.c_int32()
    assert lib.spgg_stat_stripes(None, ctypes.byref(n)) == _lib.E_ARG
    assert lib.spgg_destroy(None) == _lib.OK


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_create_failures_report_a_reason(monkeypatch):
    """spgg_create refuses bad configurations before any device call and says why through
    spgg_last_error(NULL); an SPGG_APT value other than 1 / max is an error, not ignored."""
    lib = _lib.load()

    def create(**kw):
        base = dict(device=0, n_rep=2, L=200, second_order=0, state_mode=_lib.STATE_REPUTATION,
                    rng_mode=_lib.RNG_PHILOX, iterations=10, rep_int8=1, algorithm=_lib.ALG_QLEARNING)
        base.update(kw)
        ctx = ctypes.c_void_p()
        rc = lib.spgg_create(ctypes.byref(ctx), _lib.Config(**base))
        assert not ctx.value
        return rc, lib.spgg_last_error(None).decode()

    rc, msg = create(batch_reps=1)
    assert rc == _lib.E_ARG and "batch_reps" in msg
    rc, msg = create(algorithm=9)
    assert rc == _lib.E_ARG and "algorithm" in msg
    monkeypatch.setenv("SPGG_TUNING", "1")
    monkeypatch.setenv("SPGG_APT", "3")
    rc, msg = create()
    assert rc == _lib.E_ARG and "SPGG_APT=3" in msg and "max" in msg
    monkeypatch.setenv("SPGG_APT", "4")   # Q-learning's maximum, not Double-Q's
    rc, msg = create(algorithm=_lib.ALG_DOUBLE_Q)
    assert rc == _lib.E_ARG and "2 agents per thread" in msg
    with pytest.raises(_lib.SpggError, match="SPGG_APT=4"):
        _lib.check(rc, None, "spgg_create")


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_library_build_id_matches_sources(tmp_path):
    """Freshness by content: the in-tree library carries the hash of the sources, flags and
    defines it was built from (spgg_build_id), and the package refuses a library whose id
    differs from the sources (build.py), whatever the file times say."""
    import shutil
    from spgg_amd import build as B
    lib = _lib.load()
    assert lib.spgg_build_id().decode() == B.build_id() == B.library_build_id(_lib.LIB_PATH)
    assert not B.needs_build()
    assert B.build_id(("SPGG_GEN_OUT=3",)) != B.build_id()     # defines are part of the id
    stale = tmp_path / "lib.so"
    data = open(_lib.LIB_PATH, "rb").read().replace(b"spgg-build:" + B.build_id().encode(),
                                                   b"spgg-build:0000000000000000")
    stale.write_bytes(data)
    assert B.needs_build(str(stale))
    assert B.library_build_id(str(stale)) == "0" * 16


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_only_documented_environment_knobs_are_read():
    """The shipped library names no timing-only knob (SPGG_TIMING, SPGG_ABLATE, generator A/B
    switches: compile-time defines of tuning builds whose results are wrong by design); every
    SPGG_* string it carries is a layout / scheduling knob documented in spgg_abi.h."""
    data = open(_lib.LIB_PATH, "rb").read()
    names = {m.decode() for m in re.findall(rb"SPGG_[A-Z0-9_]+", data)}
    for bad in ("SPGG_TIMING", "SPGG_ABLATE", "SPGG_STAMPS", "SPGG_GEN_ABLATE", "SPGG_GEN_NR", "SPGG_GEN_OUT",
                "SPGG_GEN_PUB", "SPGG_GEN_SETPRIO", "SPGG_GEN_VGPR"):
        assert bad not in names, bad
    header = open(HEADER).read()
    knobs = header[header.index("Environment knobs"):header.index("int spgg_create")]
    undocumented = sorted(n for n in names if n not in knobs)
    assert not undocumented, undocumented


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")
def test_tuning_knobs_need_the_tuning_switch(monkeypatch):
    """Without SPGG_TUNING=1 the library ignores its tuning knobs: an SPGG_APT or SPGG_TILE
    left in a user's environment changes nothing (here: a value that would fail spgg_create
    is not even read, and the tile is the planner's)."""
    lib = _lib.load()
    base = dict(device=0, n_rep=2, L=200, second_order=0, state_mode=_lib.STATE_REPUTATION,
                rng_mode=_lib.RNG_PHILOX, iterations=10, rep_int8=1, algorithm=_lib.ALG_QLEARNING)
    monkeypatch.delenv("SPGG_TUNING", raising=False)
    monkeypatch.setenv("SPGG_APT", "3")
    monkeypatch.setenv("SPGG_TILE", "16x16")
    ctx = ctypes.c_void_p()
    rc = lib.spgg_create(ctypes.byref(ctx), _lib.Config(**base))
    if rc == _lib.E_HIP:   # no device in this container: creation stops at hipSetDevice
        assert "SPGG_APT" not in lib.spgg_last_error(None).decode()
        return
    assert rc == _lib.OK
    tw, th = ctypes.c_int32(), ctypes.c_int32()
    assert lib.spgg_tile_shape(ctx, ctypes.byref(tw), ctypes.byref(th)) == _lib.OK
    assert (tw.value, th.value) != (16, 16)
    lib.spgg_destroy(ctx)
