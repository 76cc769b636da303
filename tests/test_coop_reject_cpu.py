"""The cooperative rejection sampler (csrc/rtw_device.hpp coop_reject_mixed,
DESIGN.md §5.7) emulated lane by lane on the CPU: for a 64-lane wave with a
mix of requests — unit-ball points (dim 3, rand.zig:22-28), lens-disk points
plus the following time draw (dim 2, rand.zig:30-36 + main.zig:99) and one
speculative dielectric draw (dim 1) — every lane gets exactly the point, the
final RNG state and the extra draw of its own sequential loop under the
Tier-B counter RNG (each draw one Weyl step through the Tier-B mixer; rare long-leading-zero
words from the draw's extension stream).  Pure Python, test infrastructure."""
import math
import random
import struct

import pytest

M64 = (1 << 64) - 1
GAMMA = 0x9E3779B97F4A7C15
EXT = 0x5851F42D4C957F2D


def mix(z):  # Tier-B mixer (oracle/rtw_oracle.c ro_tb_mix): four Feistel half-rounds
    hi, lo = z >> 32, z & 0xFFFFFFFF
    for i, m in enumerate((0xD2511F53, 0xCD9E8D57, 0x9E3779B1, 0x85EBCA6B)):
        if i % 2 == 0:
            t = hi * m
            lo ^= t >> 32
            hi = t & 0xFFFFFFFF
        else:
            t = lo * m
            hi ^= t >> 32
            lo = t & 0xFFFFFFFF
    return (hi << 32) | lo


def clz64(v):
    return 64 - v.bit_length()


def rnd(st):
    """Random.float(f64) of the draw after state st -> (value, new state)."""
    st = (st + GAMMA) & M64
    v = mix(st)
    lz = clz64(v)
    if lz >= 12:  # the draw's own extension stream (rtw_device.hpp f64_long_lz)
        e, lz = st ^ EXT, 12
        while True:
            e = (e + GAMMA) & M64
            addl = clz64(mix(e))
            lz += addl
            if addl != 64:
                break
            if lz >= 1022:
                lz = 1022
                break
    bits = ((1022 - lz) << 52) | (v & ((1 << 52) - 1))
    return struct.unpack("<d", struct.pack("<Q", bits))[0], st


def m11(r):
    return r * 2.0 - 1.0  # fma(r, 2, -1): r*2 is exact


def in_ball(dim, x0, x1, x2):
    if dim == 3:
        return not (x0 * x0 + x1 * x1 + x2 * x2 >= 1.0)
    return not (x0 * x0 + x1 * x1 + 0.0 * 0.0 >= 1.0)


def sequential(dim, st):
    """The lane's own loop: (point, state after it, the extra draw)."""
    if dim == 0:
        return None, st, None
    if dim == 1:
        r, _ = rnd(st)
        return None, st, r
    while True:
        x = []
        for _ in range(dim):
            r, st = rnd(st)
            x.append(m11(r))
        if in_ball(dim, x[0], x[1], x[2] if dim == 3 else 0.0):
            break
    extra = rnd(st)[0] if dim == 2 else None  # the sample's time draw
    return tuple(x), st, extra


def coop(dims, states):
    """Lane-by-lane emulation of coop_reject_mixed for one wave."""
    n = len(dims)
    st = list(states)
    x = [None] * n
    raw = [None] * n
    pending = [False] * n
    for l in range(n):  # round 0: own first candidate (three draws, SIMT)
        if dims[l] == 0:
            continue
        s = st[l]
        r0, s = rnd(s)
        r1, s = rnd(s)
        s2 = s
        r2, s = rnd(s)
        x[l] = (m11(r0), m11(r1), m11(r2))
        raw[l] = r0 if dims[l] == 1 else r2
        st[l] = s if dims[l] == 3 else (s2 if dims[l] == 2 else st[l])
        pending[l] = dims[l] >= 2 and not in_ball(dims[l], *x[l])
    nextq = [0] * n
    rounds = 0
    while any(pending):
        rounds += 1
        P = [l for l in range(n) if pending[l]]
        m = len(P)
        lc = int(math.log2(64 // m))  # c = 2^lc candidates per pending lane
        c = 1 << lc
        slots = [(st[l], nextq[l], dims[l]) for l in P]  # by rank
        results = {}
        for lane in range(64):  # every lane of the wave evaluates one candidate
            orank = lane >> lc
            if orank >= m:
                continue
            B, q0, d = slots[orank]
            s = (B + d * (q0 + (lane & (c - 1))) * GAMMA) & M64
            ya, s = rnd(s)
            yb, s = rnd(s)
            yr, s = rnd(s)
            y = (m11(ya), m11(yb), m11(yr))
            results[lane] = (in_ball(d, *y), y, yr)
        for rank, l in enumerate(P):
            first = (rank << lc) & 63
            mine = [j for j in range(c) if results.get(first + j, (False,))[0]]
            if mine:
                jj = mine[0]
                _, y, yr = results[first + jj]
                x[l], raw[l] = y, yr
                st[l] = (st[l] + dims[l] * (nextq[l] + jj + 1) * GAMMA) & M64
                pending[l] = False
            else:
                nextq[l] += c
    return x, st, raw, rounds


@pytest.mark.parametrize("seed,mode", [(1, "mixed"), (2, "mixed"), (3, "balls"), (4, "disks"), (5, "one"),
                                       (6, "mixed"), (7, "mixed"), (8, "dense")])
def test_coop_reject_mixed_matches_sequential_loops(seed, mode):
    g = random.Random(seed)
    for _ in range(40):
        if mode == "balls":
            dims = [3] * 64
        elif mode == "disks":
            dims = [2] * 64
        elif mode == "one":  # a single requesting lane: it gets all 64 lanes' candidates
            dims = [0] * 64
            dims[g.randrange(64)] = g.choice([2, 3])
        elif mode == "dense":
            dims = [g.choice([2, 3]) for _ in range(64)]
        else:
            dims = [g.choice([0, 1, 2, 3, 3, 2]) for _ in range(64)]
        states = [g.getrandbits(64) for _ in range(64)]
        x, st, raw, _ = coop(dims, states)
        for l in range(64):
            px, pst, pextra = sequential(dims[l], states[l])
            assert st[l] == pst, (l, dims[l])
            if dims[l] >= 2:
                assert x[l][:dims[l]] == px, (l, dims[l])
            if dims[l] == 2 or dims[l] == 1:
                assert raw[l] == pextra, (l, dims[l])


def test_rare_long_leading_zero_draw_uses_the_extension_stream():
    # A state whose next word has >= 12 leading zeros exercises the extension
    # branch; the counter rule makes it addressable from any lane.
    g = random.Random(11)
    for _ in range(200000):
        s = g.getrandbits(64)
        if clz64(mix((s + GAMMA) & M64)) >= 12:
            break
    else:
        pytest.skip("no long-leading-zero word found")
    r, s2 = rnd(s)
    assert s2 == (s + GAMMA) & M64 and 0.0 <= r < 2.0 ** -12
