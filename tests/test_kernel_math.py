"""CPU emulation of crc64.hip's arithmetic, checked against the oracle.

The kernel never runs here; this pins the math it is built on so a GPU mismatch can
only come from the device code itself:
  * the reversed-domain slice-by-4 tables R_j = bswap(T_j) and their LDS image
    (Tab4::src_index: 16 replicas, tables paired per 16-B slot), addressed exactly as
    Tab4::step4 / step1 build addresses with v_perm, for every lane of a wave;
  * the quad transpose (two DPP quad_perm butterfly stages) that turns quad-coalesced
    loads back into per-segment 16-B pieces;
  * the x^(8n) power tables and the segment/piece combination of entries.
"""
import random

import pytest

M64 = (1 << 64) - 1
POLY = 0x42F0E1EBA9EA3693


def bswap64(v):
    return int.from_bytes(v.to_bytes(8, "little"), "big")


def tables():
    t = [[0] * 256 for _ in range(4)]
    for i in range(256):
        c = i << 56
        for _ in range(8):
            c = ((c << 1) ^ POLY) & M64 if c >> 63 else (c << 1) & M64
        t[0][i] = c
    for j in range(1, 4):
        for i in range(256):
            t[j][i] = t[0][t[j - 1][i] >> 56] ^ ((t[j - 1][i] << 8) & M64)
    return [[bswap64(x) for x in tj] for tj in t]


R = tables()  # R[j][i] = bswap(T_j[i]), engine.hip build_tables


def src_index(w):
    """Tab4::src_index: LDS word w = (k>>1)<<13 | index<<5 | replica<<1 | (k&1)."""
    return (((w >> 13) << 1) | (w & 1)) * 256 + ((w >> 5) & 255)


LDS = [R[i // 256][i % 256] for i in (src_index(w) for w in range(16384))]  # 128 KiB image


def v_perm(s0, s1, sel):
    """v_perm_b32: byte i of the result = byte sel.b_i of {s0:s1} (s1 = bytes 0-3), 0x0C = 0."""
    src = (s0 << 32) | s1
    out = 0
    for i in range(4):
        b = (sel >> (8 * i)) & 0xFF
        v = 0 if b == 0x0C else (src >> (8 * b)) & 0xFF
        out |= v << (8 * i)
    return out


class Tab4Emul:
    """Tab4 for one lane: per-lane table constants lc[i] and byte swizzle."""

    def __init__(self, lane):
        sw = (lane >> 4) & 1
        self.lc = []
        for i in range(4):
            k = 3 - (i ^ sw)
            self.lc.append(((lane & 15) << 4) | ((k & 1) << 3) | ((k >> 1) << 16))
        self.swz = 0x02030001 if sw else 0x03020100

    @staticmethod
    def lds(addr):
        assert addr % 8 == 0 and addr < 131072
        return LDS[addr // 8]

    def step4(self, r):
        lo, hi = r & 0xFFFFFFFF, r >> 32
        x = v_perm(lo, lo, self.swz)
        t = [self.lds(v_perm(self.lc[i], x, 0x0C060004 | (i << 8))) for i in range(4)]
        return (r >> 32) ^ t[0] ^ t[1] ^ t[2] ^ t[3]

    def step1(self, r, b):
        lc0 = self.lc[0] & 0xF0
        t0 = self.lds(v_perm(lc0, (r ^ b) & 0xFFFFFFFF, 0x0C060004))
        return (r >> 8) ^ t0

    def crc(self, data, r=0):
        """hash_global's order: bytes to 16-B alignment (relative to the start), 16-B
        steps as 2 x step8 (= 2 x step4 each), byte tail."""
        p, n = 0, len(data)
        while p + 16 <= n:
            for h in (0, 8):
                r ^= int.from_bytes(data[p + h:p + h + 8], "little")
                r = self.step4(self.step4(r))
            p += 16
        while p < n:
            r = self.step1(r, data[p])
            p += 1
        return r


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


def test_slice4_tables_are_byte_steps():
    """R_j[i] = (i shifted through j+1 byte steps of the reversed-domain CRC64)."""
    def byte_step(r, b):
        return R[0][(r ^ b) & 0xFF] ^ (r >> 8)
    for j in range(4):
        for i in (0, 1, 0x80, 0xFF, 0x5A):
            r = i
            for _ in range(j + 1):
                r = byte_step(r, 0)
            assert R[j][i] == r, (j, i)


@pytest.mark.parametrize("lane", [0, 1, 15, 16, 17, 31, 32, 47, 48, 63])
def test_step4_lane_addressing_matches_oracle(oracle, lane):
    """Every lane class (replica, swapped table pair) reaches the same CRC."""
    rng = random.Random(lane)
    tb = Tab4Emul(lane)
    for n in (0, 1, 7, 15, 16, 17, 33, 64, 255, 1000):
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert bswap64(tb.crc(d)) == oracle.crc64(d), (lane, n)


def test_swapped_lanes_hit_opposite_table_halves():
    """Lanes l and l+16 read the two 8-B halves of one 16-B LDS slot in the same
    instruction (the conflict-free pairing of ds_read_b64 half-waves)."""
    for lane in range(16):
        a, b = Tab4Emul(lane), Tab4Emul(lane + 16)
        for i in range(4):
            assert (a.lc[i] ^ b.lc[i]) == 8, (lane, i)
            assert (a.lc[i] >> 4) & 0xF == lane


def test_step1_continues_a_running_register(oracle):
    rng = random.Random(2)
    d = bytes(rng.getrandbits(8) for _ in range(77))
    tb = Tab4Emul(21)
    r = 0
    for b in d[:5]:
        r = tb.step1(r, b)
    assert bswap64(tb.crc(d[5:], r)) == oracle.crc64(d)


def quad_transpose_emul(regs):
    """regs[m][o]: lane m's register o. DPP quad_perm xor1 / xor2 butterflies (quad_stage)."""
    def stage(regs, lo_i, hi_i, bitpos):
        x = 1 << bitpos
        new = [list(r) for r in regs]
        for m in range(4):
            bit = (m >> bitpos) & 1
            plo, phi = regs[m ^ x][lo_i], regs[m ^ x][hi_i]
            new[m][hi_i] = regs[m][hi_i] if bit else plo
            new[m][lo_i] = phi if bit else regs[m][lo_i]
        return new
    regs = stage(regs, 0, 1, 0)
    regs = stage(regs, 2, 3, 0)
    regs = stage(regs, 0, 2, 1)
    regs = stage(regs, 1, 3, 1)
    return regs


def test_quad_transpose_restores_segment_pieces():
    """Load q of quad lane m reads piece m (16 B at 16m) of owner q's segment; after the
    transpose lane m's register j holds piece j of its own segment."""
    loaded = [[("owner", q, "piece", m) for q in range(4)] for m in range(4)]
    out = quad_transpose_emul(loaded)
    for m in range(4):
        assert out[m] == [("owner", m, "piece", j) for j in range(4)]


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
