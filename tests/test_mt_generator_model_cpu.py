"""A model check of the MT19937 draw generator's wave protocol (csrc/spgg_kernels.hip,
spgg_mt_gen_kernel) on the CPU: the recurrence and output waves are restated as coroutines
that yield at every LDS access, run under random interleavings over a sequentially
consistent LDS, and their outputs are compared with numpy's RandomState stream.

What it checks is the kernel's index arithmetic (the contiguous 227-word ring blocks and their
mirror, the slot positions gen_slot_* with the spare lanes duplicating real ones, gen_word_pos,
the output waves' stepped ring position per chunk, the key-block bookkeeping of multi-iteration
launches) and its synchronisation (gen_done progress, gen_need flow control per batch of
chunks, the recurrence waves' block-of-slack rule), independent of timing.  The hardware ordering the
kernel relies on beyond sequential consistency (a flag store waits for the wave's earlier LDS
writes) is exercised by the -m gpu tests.  (A padding-position bug of the first version of
this kernel -- slot 3's spare lanes overwriting slot 1's words -- is the kind of defect this
finds: it failed every interleaving here and only some runs on the GPU.)"""
import random

import numpy as np
import pytest

NB, P, MB = 16, 227, 227        # kGenNB, kGenPitch, kMtBlock
RING_WORDS = P * NB             # kGenRingWords
RING = RING_WORDS + P           # + the mirror of block 0
U_BATCH = 4                     # kGenU


def word_pos(k):                 # gen_word_pos
    return (k + RING_WORDS - 624) % RING_WORDS


SLOT_BASE, SLOT_LEN = (0, 169, 58, 122), (58, 58, 64, 47)   # gen_slot_*


def position(s, lane):           # gen_position: spare lanes duplicate lane - len of their slot
    return SLOT_BASE[s] + (lane if lane < SLOT_LEN[s] else lane - SLOT_LEN[s])


def temper(y):
    y ^= y >> 11
    y ^= (y << 7) & 0x9D2C5680
    y ^= (y << 15) & 0xEFC60000
    y ^= y >> 18
    return y & 0xFFFFFFFF


def mt_next(far, a, b):
    y = (a & 0x80000000) | (b & 0x7FFFFFFF)
    return (far ^ (y >> 1) ^ (0x9908B0DF if b & 1 else 0)) & 0xFFFFFFFF


def plane_word0(n, p):
    return n * (p // 2 * 3 + (p & 1) * 2)


def run_model(n, planes, t0, t1, key, pos0, seed, NR=1, NOUT=7, PUB=4):
    rnd = random.Random(seed)
    SPW = 4 // NR
    ring = [0] * RING
    for i in range(624):
        ring[word_pos(i)] = key[i]
    gen_done = [0] * NR
    gen_need = [0] * NOUT
    W = plane_word0(n, planes) if planes % 2 == 0 else n * (planes // 2 * 3 + 2)
    E_last = pos0 + (t1 - t0 + 1) * W
    target_last = ((E_last - 1) // 624) * 624 + 624
    nblk = (target_last - 624 + MB - 1) // MB if target_last > 624 else 0
    out, keys = {}, {}

    def rec(r):
        lanes = [(i, lane, position(r * SPW + i, lane)) for i in range(SPW) for lane in range(64)]
        prev = {(i, l): ring[j + (NB - 1) * P] for i, l, j in lanes}
        ca = {(i, l): ring[j + 57 + (NB - 3) * P] for i, l, j in lanes}
        cb = {(i, l): ring[j + 58 + (NB - 3) * P] for i, l, j in lanes}
        yield
        E = pos0 + W
        mb = ((E - 1) // 624) * 624
        target = mb + 624
        lim = mind = b = 0
        t = t0
        key_mb, key_pos = 0, pos0

        def retire():
            nonlocal t, E, mb, target, key_mb, key_pos
            keys[t] = ([ring[word_pos(mb + i)] for i in range(624)], E - mb)
            key_mb, key_pos = mb, E - mb
            t += 1
            E += W
            mb = ((E - 1) // 624) * 624
            target = mb + 624

        while b != nblk:
            while NR > 1 and mind + 1 < b:
                mind = min(gen_done)
                yield
            if r == 0:
                while t <= t1 and 624 + MB * mind >= target:
                    retire()
                    yield
            F = 624 + MB * b
            while F > lim:
                m = min(gen_need)
                lim = 0xFFFFFFFF if m > 0xFFFFFFFF - (NB - 1) * MB else m + (NB - 1) * MB
                yield
            U = b % NB
            rb = ((U + 1 + NB - 3) % NB) * P
            na = {(i, l): ring[j + 57 + rb] for i, l, j in lanes}
            nb_ = {(i, l): ring[j + 58 + rb] for i, l, j in lanes}
            yield
            for i, l, j in lanes:
                x = mt_next(prev[i, l], ca[i, l], cb[i, l])
                prev[i, l] = x
                ring[j + U * P] = x
                if U == 0:
                    ring[j + NB * P] = x
                ca[i, l], cb[i, l] = na[i, l], nb_[i, l]
            yield
            b += 1
            if NR > 1 or (U + 1) % PUB == 0:
                gen_done[r] = b
            yield
            mind = min(gen_done) if NR > 1 else b
        gen_done[r] = b
        if r != 0:
            return
        while mind < nblk:
            mind = min(gen_done)
            yield
        while t <= t1:
            retire()

    def outw(ow):
        nchunk = (n + 63) // 64
        kpos, seen = pos0, 624
        for t in range(t0, t1 + 1):
            for p in range(planes):
                dbl = (p & 1) == 0
                wmul = 2 if dbl else 1
                cstep = 64 * wmul * NOUT
                first = kpos + plane_word0(n, p) + 64 * wmul * ow
                rpos = word_pos(first)                    # stepped per chunk, never divided
                for c in range(ow, nchunk, NOUT * U_BATCH):
                    nb = min(U_BATCH, (nchunk - 1 - c) // NOUT + 1)
                    cl = c + (nb - 1) * NOUT
                    last = first + cstep * (nb - 1) + wmul * min(64, n - 64 * cl) - 1
                    gen_need[ow] = first                  # the batch's first word, once per batch
                    yield
                    while seen <= last:
                        seen = 624 + MB * min(gen_done)
                        yield
                    rp = rpos
                    for u in range(nb):
                        cu = c + u * NOUT
                        cnt = min(64, n - 64 * cu)
                        assert rp == word_pos(first + cstep * u)
                        if dbl:
                            out[t, p, cu] = [(temper(ring[rp + 2 * l]), temper(ring[rp + 2 * l + 1]))
                                             for l in range(cnt)]
                        else:
                            out[t, p, cu] = [temper(ring[rp + l]) for l in range(cnt)]
                        rp += cstep
                        rp -= RING_WORDS if rp >= RING_WORDS else 0
                        yield
                    rpos += cstep * nb
                    rpos -= RING_WORDS if rpos >= RING_WORDS else 0
                    first += cstep * nb
            kpos += W
        gen_need[ow] = 0xFFFFFFFF

    waves = [rec(r) for r in range(NR)] + [outw(w) for w in range(NOUT)]
    alive = list(range(len(waves)))
    while alive:
        i = rnd.choice(alive)
        try:
            next(waves[i])
        except StopIteration:
            alive.remove(i)
    return out, keys


@pytest.mark.parametrize("NOUT", [3, 7, 1])
@pytest.mark.parametrize("n,planes", [(100, 2), (576, 2), (300, 6), (250, 3), (1000, 2)])
def test_generator_protocol_model(NOUT, n, planes):
    T = 4
    for seed in range(2):
        rs = np.random.RandomState(seed + 11)
        rs.uniform(size=(seed * 37) % 500)          # start mid-block (pos != 624)
        st = rs.get_state()
        key, pos = [int(x) for x in st[1]], int(st[2])
        out, keys = run_model(n, planes, 1, T, key, pos, seed, NOUT=NOUT)
        W = n * (planes // 2 * 3 + (planes & 1) * 2)
        nchunk = (n + 63) // 64
        for t in range(1, T + 1):
            words = rs.randint(0, 2 ** 32, size=W, dtype=np.uint64)   # the raw 32-bit outputs
            for p in range(planes):
                base = plane_word0(n, p)
                for c in range(nchunk):
                    cnt = min(64, n - 64 * c)
                    if p % 2 == 0:
                        want = [(int(words[base + 128 * c + 2 * l]), int(words[base + 128 * c + 2 * l + 1]))
                                for l in range(cnt)]
                    else:
                        want = [int(words[base + 64 * c + l]) for l in range(cnt)]
                    assert out[t, p, c] == want, (seed, t, p, c)
            k, ps = keys[t]
            s = rs.get_state()
            assert ps == int(s[2]) and k == [int(x) for x in s[1]], (seed, t)


def test_slot_positions_cover_the_block():
    """The real lanes own the 227 positions once each; each of the 29 spare lanes duplicates a
    real lane OF ITS OWN SLOT (the same instruction: same position, operands and previous word,
    so the same value written to the same address -- a spare lane of another slot or wave
    writing a real position would race its owner)."""
    real = [position(s, lane) for s in range(4) for lane in range(SLOT_LEN[s])]
    assert sorted(real) == list(range(MB))
    for s in range(4):
        own = {position(s, lane) for lane in range(SLOT_LEN[s])}
        assert {position(s, lane) for lane in range(SLOT_LEN[s], 64)} <= own
    # slots 0 and 1 (one wave) hold positions 0-57 and 169-226: the positions that need the
    # block two back read only that wave's own words
    assert {position(0, l) for l in range(58)} == set(range(58))
    assert {position(1, l) for l in range(58)} == set(range(169, 227))
