"""CPU emulation of crc64.hip's arithmetic, checked against the oracle.

The kernel never runs here; this pins the math it is built on (reversed-domain
slice-by-2 tables, x^(8n) power tables, flat segments + piece combination) so a
GPU mismatch can only come from the device code itself.
"""
import random

import pytest

M64 = (1 << 64) - 1
POLY = 0x42F0E1EBA9EA3693


def bswap64(v):
    return int.from_bytes(v.to_bytes(8, "little"), "big")


def tables():
    t0 = []
    for i in range(256):
        c = i << 56
        for _ in range(8):
            c = ((c << 1) ^ POLY) & M64 if c >> 63 else (c << 1) & M64
        t0.append(c)
    t1 = [t0[t0[i] >> 56] ^ ((t0[i] << 8) & M64) for i in range(256)]
    return [bswap64(x) for x in t0], [bswap64(x) for x in t1]


R0, R1 = tables()


def mulmod(a, b):
    r = 0
    for i in range(63, -1, -1):
        r = ((r << 1) ^ POLY) & M64 if r >> 63 else (r << 1) & M64
        if (b >> i) & 1:
            r ^= a
    return r


def xpow8(n):
    """x^(8n) mod G via the power tables' factorisation (one factor per set bit)."""
    k, r, t = 0x100, 1, 0
    while n:
        if n & 1:
            r = mulmod(r, k)
        k = mulmod(k, k)
        n >>= 1
        t += 1
    return r


def crc_range_emul(data: bytes) -> int:
    """Exactly the step sequence of crc_range(): byte head, 8-byte words as 4 x step2, tail."""
    r = 0
    p = 0
    n = len(data)

    def step2(r):
        return (r >> 16) ^ R1[r & 0xFF] ^ R0[(r >> 8) & 0xFF]

    def step1(r, b):
        return R0[(r ^ b) & 0xFF] ^ (r >> 8)

    while p + 8 <= n:
        r ^= int.from_bytes(data[p:p + 8], "little")
        for _ in range(4):
            r = step2(r)
        p += 8
    while p + 2 <= n:
        r ^= data[p] | (data[p + 1] << 8)
        r = step2(r)
        p += 2
    if p < n:
        r = step1(r, data[p])
    return bswap64(r)


def test_slice2_matches_oracle(oracle):
    rng = random.Random(1)
    for n in list(range(0, 40)) + [255, 256, 1000, 4097]:
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert crc_range_emul(d) == oracle.crc64(d), n


def test_head_bytes_then_words(oracle):
    # unaligned head handled byte-serially, then words: same register
    rng = random.Random(2)
    d = bytes(rng.getrandbits(8) for _ in range(77))

    def step1(r, b):
        return R0[(r ^ b) & 0xFF] ^ (r >> 8)

    r = 0
    for b in d[:5]:
        r = step1(r, b)
    rest = d[5:]
    # continue with the word loop from state r
    p = 0
    while p + 8 <= len(rest):
        r ^= int.from_bytes(rest[p:p + 8], "little")
        for _ in range(4):
            r = (r >> 16) ^ R1[r & 0xFF] ^ R0[(r >> 8) & 0xFF]
        p += 8
    for b in rest[p:]:
        r = step1(r, b)
    assert bswap64(r) == oracle.crc64(d)


def test_shift_combination(oracle):
    """crc(A||B) = crc(A) * x^(8|B|) mod G  ^  crc(B)   (init 0, xorout 0)."""
    rng = random.Random(3)
    for la, lb in [(1, 1), (7, 300), (1024, 1024), (13, 4096), (0, 5), (5, 0)]:
        a = bytes(rng.getrandbits(8) for _ in range(la))
        b = bytes(rng.getrandbits(8) for _ in range(lb))
        assert mulmod(oracle.crc64(a), xpow8(lb)) ^ oracle.crc64(b) == oracle.crc64(a + b)


def test_byte_tables_for_shift():
    """shift[t][k][i] tables reproduce mulmod(c, x^(8*2^t)) byte-wise."""
    rng = random.Random(4)
    K = 0x100
    for t in range(6):
        tab = [[mulmod(i << (8 * k), K) for i in range(256)] for k in range(8)]
        for _ in range(20):
            c = rng.getrandbits(64)
            v = 0
            for k in range(8):
                v ^= tab[k][(c >> (8 * k)) & 0xFF]
            assert v == mulmod(c, K)
        K = mulmod(K, K)


@pytest.mark.parametrize("seg", [16, 64, 256])
def test_segment_piece_combination(oracle, seg):
    """Flat segments + per-entry pieces (the kernel's work split) give the entry CRCs."""
    rng = random.Random(seg)
    lens = [rng.choice([0, 1, 3, 17, seg - 1, seg, seg + 1, 3 * seg + 5]) for _ in range(60)]
    base = 11
    offs = [base]
    for L in lens:
        offs.append(offs[-1] + L)
    total = offs[-1] - base
    payload = bytes(rng.getrandbits(8) for _ in range(offs[-1] + 3))
    nseg = max(1, -(-total // seg))
    acc = {}
    out = {}
    for k in range(nseg):
        s0 = base + k * seg
        s1 = base + total if k + 1 == nseg else s0 + seg
        for e in range(len(lens)):
            a, b = offs[e], offs[e + 1]
            if a == b:
                if (s0 <= a < s1) or (k + 1 == nseg and a == s1):
                    out[e] = 0
                continue
            lo, hi = max(a, s0), min(b, s1)
            if lo >= hi:
                continue
            c = mulmod(oracle.crc64(payload[lo:hi]), xpow8(b - hi))
            acc[e] = acc.get(e, 0) ^ c
    for e, v in acc.items():
        out[e] = v
    for e in range(len(lens)):
        assert out[e] == oracle.crc64(payload[offs[e]:offs[e + 1]]), e
