"""MT19937 jump-ahead (csrc/spgg_mt.hip), host side: the library's g = x^e mod phi, applied
as the device jump kernel applies it, moves a window of numpy's own MT19937 stream forward
by exactly D words.

The stream is numpy.random.RandomState's (the reference's global RNG, algorithms.py:105,108):
its raw words are extended here with the MT19937 recurrence and checked against numpy's
output (tempered words, randint(0, 2**32, dtype=uint32) = one word each), so the property
is pinned on the reference's generator, not on a restatement of it."""
import ctypes
import os

import numpy as np
import pytest

from spgg_amd import _lib

pytestmark = pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libspgg_hip.so not built")


def _temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def _stream(key, count):
    """Raw words x[0 .. count) with x[0..623] = key: x[k+624] = x[k+397] ^ twist(x[k], x[k+1])."""
    x = np.zeros(max(count, 624), dtype=np.uint32)
    x[:624] = key
    k = 624
    while k < count:  # 227 words per step depend only on words >= 227 back
        m = np.arange(k, min(k + 227, count))
        lo_k, lo_k1, far = x[m - 624], x[m - 623], x[m - 227]
        y = (lo_k & np.uint32(0x80000000)) | (lo_k1 & np.uint32(0x7FFFFFFF))
        x[m] = far ^ (y >> np.uint32(1)) ^ np.where(lo_k1 & np.uint32(1), np.uint32(0x9908B0DF), np.uint32(0))
        k += 227
    return x[:count]


def _poly(e):
    lib = _lib.load()
    g = np.zeros(624, dtype=np.uint32)
    assert lib.spgg_mt_jump_poly(ctypes.c_int64(e), g.ctypes.data) == 0
    bits = np.unpackbits(g.view(np.uint8), bitorder="little")
    assert not bits[19937:].any()  # degree < 19937
    return np.flatnonzero(bits)


def test_stream_is_numpys():
    rs = np.random.RandomState(12345)
    _, key, pos, _, _ = rs.get_state()
    assert pos == 624
    x = _stream(np.asarray(key, dtype=np.uint32), 624 + 5000)
    assert np.array_equal(_temper(x[624:]), rs.randint(0, 2 ** 32, size=5000, dtype=np.uint32))


@pytest.mark.parametrize("D", [1, 2, 227, 624, 1000, 19937, 120000, 1_000_003])
def test_jump_moves_a_window_by_D(D):
    rs = np.random.RandomState(D % 1000)
    rs.randint(0, 2, size=D % 777)            # some state mid-block
    key = np.asarray(rs.get_state()[1], dtype=np.uint32)
    B = 37                                    # window start, not block aligned
    x = _stream(key, B + D + 624)
    idx = _poly(D - 1)
    j = np.arange(624)
    got = np.bitwise_xor.reduce(x[B + 1 + idx[:, None] + j[None, :]], axis=0)
    want = x[B + D: B + D + 624]
    if D == 1:   # x^0 = 1: X[B+1+j]
        assert np.array_equal(got, x[B + 1: B + 625])
    assert np.array_equal(got, want)


def test_jump_ignores_the_low_bits_of_the_window_start():
    """Only the top bit of x[B] is state: a window whose first word's low 31 bits are
    garbage jumps to the same words (the device never needs x[B] exact)."""
    rs = np.random.RandomState(7)
    key = np.asarray(rs.get_state()[1], dtype=np.uint32)
    D = 50_000
    x = _stream(key, D + 624)
    y = x.copy()
    y[0] ^= np.uint32(0x7FFFFFFF)
    y = _stream(y[:624], D + 624)
    assert np.array_equal(x[D:], y[D:])
    idx = _poly(D - 1)
    got = np.bitwise_xor.reduce(y[1 + idx[:, None] + np.arange(624)[None, :]], axis=0)
    assert np.array_equal(got, x[D:D + 624])


def test_powers_compose():
    """x^(a+b) = x^a * x^b mod phi, seen through the stream: jumping D1 then D2 lands where
    one jump of D1 + D2 does."""
    rs = np.random.RandomState(99)
    key = np.asarray(rs.get_state()[1], dtype=np.uint32)
    D1, D2 = 30_001, 44_444
    x = _stream(key, D1 + D2 + 624)
    j = np.arange(624)
    w1 = np.bitwise_xor.reduce(x[1 + _poly(D1 - 1)[:, None] + j[None, :]], axis=0)
    y = _stream(w1, D2 + 624)
    w2 = np.bitwise_xor.reduce(y[1 + _poly(D2 - 1)[:, None] + j[None, :]], axis=0)
    assert np.array_equal(w2, x[D1 + D2: D1 + D2 + 624])


def test_tempered_low_bit_is_a_parity_of_raw_bits():
    """randint(0, 2) is the tempered word's bit 0; the generator computes it as the parity of
    raw bits 0, 3, 14, 18, 22, 29 (spgg_kernels.hip kTemperBit0)."""
    y = np.random.RandomState(0).randint(0, 2 ** 32, size=200_000, dtype=np.uint32)
    z = y & np.uint32(0x20444009)
    par = np.zeros_like(z)
    for b in range(32):
        par ^= (z >> np.uint32(b)) & np.uint32(1)
    assert np.array_equal(_temper(y) & np.uint32(1), par)


def test_doubled_jumps_derived_by_squaring():
    """The generator's jump levels D << j (polynomial exponents 2e + 1 of the level below) are
    derived from the cached level by one squaring and one multiplication by x
    (spgg_mt.hip jump_poly); each still moves a window by exactly its distance."""
    rs = np.random.RandomState(2024)
    key = np.asarray(rs.get_state()[1], dtype=np.uint32)
    D = 12_347
    x = _stream(key, (D << 2) + 624 + 1)
    j = np.arange(624)
    for lvl in range(3):          # level 0 exponentiated, levels 1 and 2 derived from it
        Dl = D << lvl
        got = np.bitwise_xor.reduce(x[1 + _poly(Dl - 1)[:, None] + j[None, :]], axis=0)
        assert np.array_equal(got, x[Dl: Dl + 624]), lvl
