"""GPU parity: libjrq CRC64 / LogEntry.checksum kernels vs the CPU oracle (bit-exact).

Oracle = oracle/jraft_oracle.c, the byte-at-a-time restatement of
jraft-core/.../util/CRC64.java:100-110 and entity/LogEntry.java:88-108,
pinned by tests/golden (catalogue check value + table digest of CRC64.java:41-92).
"""
import json
import os

import numpy as np
import pytest

from jraft_amd import _lib
from jraft_amd import workloads as W
from devio import to_dev, host_np

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _bytes_batch(items):
    offs = [0]
    for b in items:
        offs.append(offs[-1] + len(b))
    return np.frombuffer(b"".join(items) or b"\0", dtype=np.uint8).copy(), np.array(offs, np.uint64)


def test_known_answers(engine):
    """CRC-64/ECMA-182 catalogue check value (CRC64.java:36-39) and derived KATs."""
    items = [b"123456789", b"hello world", b"", b"a"]
    payload, offs = _bytes_batch(items)
    got = engine.crc64_batch(payload, offs)
    assert [int(x) for x in got] == [0x6C40DF5F0B497347, 0x12511F272D9BC22A, 0, int(got[3])]


def test_golden_crc_vectors(engine):
    with open(os.path.join(GOLDEN, "crc64_vectors.json")) as f:
        g = json.load(f)
    payload = np.frombuffer(bytes.fromhex(g["payload_hex"]), dtype=np.uint8).copy()
    offs = np.array(g["offsets"], dtype=np.uint64)
    got = engine.crc64_batch(payload, offs)
    assert [f"0x{int(x):016X}" for x in got] == g["crc64"]


@pytest.mark.parametrize("n,max_len,start", [(1, 1, 0), (7, 33, 5), (64, 300, 0), (1000, 5000, 3),
                                             (20000, 700, 0), (3000, 70000, 17)])
def test_ragged_batches(engine, oracle, n, max_len, start):
    offs = W.ragged_offsets(1000 + n, n, max_len, start=start)
    payload = W.random_bytes(n, int(offs[-1]) + 5)
    got = engine.crc64_batch(payload, offs)
    exp = oracle.crc64_batch(payload, offs)
    np.testing.assert_array_equal(got, exp)


def test_all_empty_entries(engine):
    offs = np.full(10, 7, dtype=np.uint64)
    got = engine.crc64_batch(np.zeros(16, np.uint8), offs)
    assert not got.any()


def test_one_huge_entry_spanning_segments(engine, oracle):
    """A 48 MiB entry is split over ~all lanes; pieces re-combine through x^(8n) shifts."""
    payload = W.random_bytes(5, (48 << 20) + 1)
    offs = np.array([1, 48 << 20], dtype=np.uint64)
    assert int(engine.crc64_batch(payload, offs)[0]) == oracle.crc64(payload[1:48 << 20].tobytes())


def test_mixed_huge_and_tiny(engine, oracle):
    lens = [3, 0, 9 << 20, 1, 0, 100, 5 << 20, 17, 0]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    payload = W.random_bytes(6, int(offs[-1]))
    np.testing.assert_array_equal(engine.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))


@pytest.mark.parametrize("seg", ["64", "100", "1000"])
def test_tiny_segments_stress_straddlers(oracle, seg):
    """Forced tiny segments: nearly every entry spans many segments, so every result goes
    through the x^(8n) shifts and the atomic last-arriver hand-off (all lanes, all XCDs)."""
    from jraft_amd import Engine
    with Engine(0) as e:
        e.debug_set(_lib.DBG_CRC_SEG_BYTES, int(seg))
        offs = W.ragged_offsets(int(seg), 20000, 3000, start=3)
        payload = W.random_bytes(int(seg), int(offs[-1]) + 1)
        exp = oracle.crc64_batch(payload, offs)
        for _ in range(3):
            np.testing.assert_array_equal(e.crc64_batch(payload, offs), exp)


@pytest.mark.parametrize("seg,seg_map", [("0", "0"), ("0", "1"), ("256", "1"), ("768", "0"),
                                         ("4096", "1"), (str(1 << 20), "0")])
def test_segment_sizes_and_maps(oracle, seg, seg_map):
    """Every segment size (rounded to 256 B) and chunk-to-workgroup map is bit-exact on
    ragged, unaligned and long entries: pieces land in per-segment slots (finish kernel)
    or go through the atomic hand-off when an entry spans more than 64 segments."""
    from jraft_amd import Engine
    lens = [0, 1, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1023, 4099, 16384, 100000, 3 << 20, 7]
    offs = np.concatenate([[5], 5 + np.cumsum(lens)]).astype(np.uint64)
    payload = W.random_bytes(11, int(offs[-1]) + 2)
    rag = W.ragged_offsets(12, 5000, 9000, start=1)
    payload2 = W.random_bytes(13, int(rag[-1]) + 1)
    with Engine(0) as e:
        e.debug_set(_lib.DBG_CRC_SEG_BYTES, int(seg))
        e.debug_set(_lib.DBG_CRC_SEG_MAP, int(seg_map))
        np.testing.assert_array_equal(e.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))
        np.testing.assert_array_equal(e.crc64_batch(payload2, rag), oracle.crc64_batch(payload2, rag))


@pytest.mark.parametrize("seg,n,lo,hi", [("256", 600, 65, 400), ("512", 600, 65, 400),
                                         ("256", 24, 4097, 12000)])
def test_adjacent_long_entries_group_slots(oracle, seg, n, lo, hi):
    """Back-to-back entries of lo..hi segments: every 64-segment group slot (and, past 4096
    segments, every 64-group supergroup slot) is shared by one long entry ending in it and
    one starting in it (multi-level hand-off keys)."""
    from jraft_amd import Engine
    S = int(seg)
    lens = W.uniform(31, n, lo * S, hi * S, stream=5)
    lens[::7] = (lo - 1) * S + 1   # exactly lo parts when aligned
    lens[3::11] = 5          # a short entry between two long ones now and then
    offs = np.concatenate([[3], 3 + np.cumsum(lens)]).astype(np.uint64)
    payload = W.random_bytes(31, int(offs[-1]) + 1)
    exp = oracle.crc64_batch(payload, offs)
    with Engine(0) as e:
        e.debug_set(_lib.DBG_CRC_SEG_BYTES, S)
        for _ in range(2):
            np.testing.assert_array_equal(e.crc64_batch(payload, offs), exp)


def test_more_segments_than_lanes(oracle):
    """256-B segments over ~90 MB: each wave loops over several chunks."""
    from jraft_amd import Engine
    offs = W.ragged_offsets(21, 40000, 4000, start=9)
    payload = W.random_bytes(21, int(offs[-1]) + 3)
    with Engine(0) as e:
        e.debug_set(_lib.DBG_CRC_SEG_BYTES, 256)
        np.testing.assert_array_equal(e.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))


def test_repeat_is_stable(engine, oracle):
    """Straddler scratch slots are re-zeroed by the last arriver: back-to-back calls agree."""
    offs = W.ragged_offsets(77, 5000, 9000)
    payload = W.random_bytes(77, int(offs[-1]))
    a = engine.crc64_batch(payload, offs)
    b = engine.crc64_batch(payload, offs)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, oracle.crc64_batch(payload, offs))


# ----------------------------------------------------------- LogEntry ---

def test_logentry_known_answers(engine, oracle):
    """LogEntryTest.testChecksum inputs (jraft-core/src/test/.../entity/LogEntryTest.java:95-125)."""
    px = oracle.peerid_checksum("localhost", 99, 1) ^ oracle.peerid_checksum("localhost", 100, 2)
    payload, offs = _bytes_batch([b"hello", b"hello", b"hEllo"])
    out = engine.logentry_checksum_batch(np.array([1, 1, 1]), np.array([100, 1, 100]),
                                         np.array([3, 3, 3]), np.array([px] * 3, np.uint64),
                                         payload, offs)
    assert [int(x) for x in out] == [0x670396DD526CA3BD, 0xF41932E9037E7E00, 0x69E2DBCC4CF8FE53]


def test_logentry_verify(engine, oracle):
    n = 4000
    offs = W.ragged_offsets(9, n, 3000)
    payload = W.random_bytes(9, int(offs[-1]))
    rng = np.random.default_rng(9)
    et = rng.integers(0, 4, n).astype(np.uint8)
    idx = rng.integers(-2**62, 2**62, n).astype(np.int64)
    term = rng.integers(0, 2**40, n).astype(np.int64)
    px = rng.integers(0, 2**63, n).astype(np.uint64) * (et == 3)
    exp = oracle.logentry_checksum_batch(et, idx, term, px, payload, offs)
    expected = exp.copy()
    bad = rng.random(n) < 0.01
    expected[bad] ^= np.uint64(1)
    has = (rng.random(n) < 0.9).astype(np.uint8)
    out, corrupt = engine.logentry_checksum_batch(et, idx, term, px, payload, offs, expected, has)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(corrupt, (bad & (has == 1)).astype(np.uint8))
    _, corrupt2 = engine.logentry_checksum_batch(et, idx, term, px, payload, offs, expected, None)
    np.testing.assert_array_equal(corrupt2, bad.astype(np.uint8))


def _entry_fields(N, seed):
    rng = np.random.default_rng(seed)
    et = rng.integers(0, 4, N).astype(np.uint8)
    idx = rng.integers(-2**62, 2**62, N).astype(np.int64)
    term = rng.integers(0, 2**40, N).astype(np.int64)
    px = rng.integers(0, 2**63, N).astype(np.uint64) * (et == 3)
    return rng, et, idx, term, px


LANES = 256 * 512  # the CRC grid's lanes on MI355X: the fixed-size kernel wants >= 1 entry each


@pytest.mark.parametrize("el,n,tail", [(256, 140000, []), (512, LANES + 5, []), (1024, LANES, [77]),
                                       (256, LANES, [0]), (768, 140000, []), (256, 4000, []),
                                       (512, 70001, []), (1024, 40000, []), (16384, 2100, []),
                                       (4096, 33000, [])])
def test_fixed_size_batches(engine, oracle, el, n, tail):
    """Host variants route batches of equal entries to the one-launch fixed-size kernel
    (crc64.hip crc64_fixed_kernel: k = 1, 2, 4 .. 64 lanes per entry combined by linearity,
    fields, verify and the store there); a ragged / zero-length tail, other lengths and small
    batches take the segment walk.
    Every result vs the oracle: LogEntry (verify, has, peers) and plain CRC."""
    lens = [el] * n + tail
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    N = len(lens)
    payload = W.random_bytes(el + n, int(offs[-1]) or 1)
    rng, et, idx, term, px = _entry_fields(N, el + n)
    exp = oracle.logentry_checksum_batch(et, idx, term, px, payload, offs)
    expected = exp.copy()
    bad = rng.random(N) < 0.02
    expected[bad] ^= np.uint64(1 << 40)
    has = (rng.random(N) < 0.8).astype(np.uint8)
    out, corrupt = engine.logentry_checksum_batch(et, idx, term, px, payload, offs, expected, has)
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(corrupt, (bad & (has == 1)).astype(np.uint8))
    out2 = engine.logentry_checksum_batch(et, idx, term, None, payload, offs)
    np.testing.assert_array_equal(out2, oracle.logentry_checksum_batch(et, idx, term, None, payload, offs))
    np.testing.assert_array_equal(engine.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))


@pytest.mark.parametrize("el,n", [(256, 140000), (512, LANES + 7), (100, 5000), (256, 3000),
                                  (16384, 8192), (16384, 8191)])
def test_fixed_dev_api(engine, oracle, el, n):
    """jrq_logentry_checksum_fixed_dev / jrq_crc64_fixed_dev (device buffers, no offsets): the
    fixed-size kernel, or the offsets path over generated offsets (100-B entries, few entries)."""
    import torch
    dev = torch.device("cuda:0")
    payload = W.random_bytes(el * 7 + n, el * n)
    offs = (np.arange(n + 1, dtype=np.uint64) * np.uint64(el))
    rng, et, idx, term, px = _entry_fields(n, el + 3 * n)
    exp = oracle.logentry_checksum_batch(et, idx, term, px, payload, offs)
    expected = exp.copy()
    bad = rng.random(n) < 0.05
    expected[bad] ^= np.uint64(3)

    def t(a):
        return to_dev(a.view(np.int64) if a.dtype == np.uint64 else a, dev)
    # a non-default torch stream shared with the engine: torch's default stream handle is 0,
    # which selects the engine's own stream (no ordering with the uploads)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        ins = [t(x) for x in (et, idx, term, px, payload, expected)]
        out = torch.zeros(n, dtype=torch.int64, device=dev)
        cor = torch.zeros(n, dtype=torch.uint8, device=dev)
        crc = torch.zeros(n, dtype=torch.int64, device=dev)
    engine.use_stream(s.cuda_stream)
    try:
        engine.logentry_checksum_fixed_dev(*ins[:5], el, out, expected=ins[5], corrupt=cor)
        engine.crc64_fixed_dev(ins[4], el, crc)
        s.synchronize()
    finally:
        engine.use_stream(None)
    np.testing.assert_array_equal(host_np(out).view(np.uint64), exp)
    np.testing.assert_array_equal(host_np(cor), bad.astype(np.uint8))
    np.testing.assert_array_equal(host_np(crc).view(np.uint64), oracle.crc64_batch(payload, offs))


def test_device_path_c1_shape(engine, oracle):
    """Device-resident variant (torch tensors, engine on its own stream), C1-shaped slice."""
    import torch
    n = 1 << 16
    b = W.entry_batch(n, 256, seed=11)
    dev = torch.device("cuda:0")
    t = {k: to_dev(v.view(np.int64) if v.dtype == np.uint64 else v, dev)
         for k, v in b.items() if isinstance(v, np.ndarray)}
    out = torch.zeros(n, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()  # the uploads went to torch's default stream; the engine uses its own
    engine.logentry_checksum_batch_dev(t["etype"], t["index"], t["term"], None, t["payload"],
                                       t["offsets"], out)
    engine.synchronize()
    exp = oracle.logentry_checksum_batch(b["etype"], b["index"], b["term"], None, b["payload"],
                                         b["offsets"])
    np.testing.assert_array_equal(host_np(out).view(np.uint64), exp)


@pytest.mark.parametrize("cfg", ["C1", "C5"])
def test_full_size_configs(engine, oracle, cfg):
    """Full BASELINE sizes (C1 256 MB, C5 1 GiB): every entry checked against the oracle."""
    c = W.CONFIGS[cfg]
    n = c["groups"] * (c["pending"] if cfg == "C1" else 1)
    b = W.entry_batch(n, c["entry_bytes"], seed=W.SEED_BASE ^ int(cfg[1]))
    got = engine.logentry_checksum_batch(b["etype"], b["index"], b["term"], None, b["payload"],
                                         b["offsets"])
    exp = oracle.logentry_checksum_batch(b["etype"], b["index"], b["term"], None, b["payload"],
                                         b["offsets"])
    np.testing.assert_array_equal(got, exp)


def test_c5_step_full_size(engine, oracle):
    """C5 as BASELINE states it, at full size: 64k regions x 3 replicas, one 16 KiB DATA entry
    per region.  The step's two halves against the oracle: LogEntry.checksum() + isCorrupted()
    over the 64k entries with 1/1024 of the stored checksums wrong (LogEntry.java:88-108,
    156-158), and the commit epoch of the 64k groups (BallotBox.commitAt replayed through real
    BallotBoxes, BallotBox.java:96-139)."""
    c = W.CONFIGS["C5"]
    n = c["groups"]
    b = W.entry_batch(n, c["entry_bytes"], seed=W.SEED_BASE ^ 5)
    exp = oracle.logentry_checksum_batch(b["etype"], b["index"], b["term"], None, b["payload"],
                                         b["offsets"])
    flip = np.zeros(n, bool)
    flip[::1024] = True
    out, corrupt = engine.logentry_checksum_batch(b["etype"], b["index"], b["term"], None,
                                                  b["payload"], b["offsets"],
                                                  expected=exp ^ flip.astype(np.uint64))
    np.testing.assert_array_equal(out, exp)
    np.testing.assert_array_equal(corrupt.astype(bool), flip)
    assert int(corrupt.sum()) == n // 1024
    q = W.quorum_batch("C5")
    committed, status = engine.quorum_epoch(q["match"], q["pending_index"], q["last_appended"],
                                            q["last_committed"], q["conf"])
    ce, se, _ = oracle.quorum_epoch_replay(q["match"], q["pending_index"], q["last_appended"],
                                           q["last_committed"], q["conf"], chunk=1024)
    np.testing.assert_array_equal(committed, ce)
    np.testing.assert_array_equal(status, se)
    assert (committed > q["last_committed"]).sum() > n // 2


# ---- streaming Checksum (RheaKV snapshot archive CRC64, §8f row 4) ----------------------------

@pytest.mark.parametrize("S,max_len,start", [(1, 1, 0), (5, 40, 3), (300, 5000, 0),
                                             (4096, 2000, 1), (2, 3_000_000, 0)])
def test_stream_update_vs_oracle(engine, oracle, S, max_len, start):
    """state[s] <- CRC64.update(chunk_s) from a nonzero register (CRC64.java:106-110)."""
    offs = W.ragged_offsets(77 + S, S, max_len, start=start)
    payload = W.random_bytes(S + 3, int(offs[-1]) + 9)
    rng = np.random.default_rng(S)
    st0 = rng.integers(0, 2**63, S, dtype=np.int64).astype(np.uint64)
    st0[0] = 0
    got = engine.crc64_stream_update(st0, payload, offs)
    exp = oracle.crc64_stream_update(st0, payload, offs)
    np.testing.assert_array_equal(got, exp)


def test_stream_archive_in_pieces(engine, oracle):
    """One 40 MB archive fed through CheckedInputStream-sized pieces (ZipUtil.java:74-94):
    the final getValue() equals CrcUtil.crc64 of the whole archive."""
    data = W.random_bytes(4242, 40 << 20)
    cuts = np.sort(np.random.default_rng(1).choice(np.arange(1, data.size), 23, replace=False))
    offs = np.concatenate([[0], cuts, [data.size]]).astype(np.uint64)
    reg = np.zeros(1, np.uint64)
    for a, b in zip(offs[:-1], offs[1:]):
        reg = engine.crc64_stream_update(reg, data, np.array([a, b], np.uint64))
    whole = engine.crc64_batch(data, np.array([0, data.size], np.uint64))
    assert int(reg[0]) == int(whole[0])
    exp = oracle.crc64_stream_update(np.zeros(1, np.uint64), data,
                                     np.array([0, data.size], np.uint64))
    assert int(reg[0]) == int(exp[0])


def test_stream_update_dev_resident_state(engine, oracle):
    """_dev variant: registers stay on the device across calls (many regions' snapshots)."""
    import torch
    S = 1000
    dev = torch.device("cuda:0")
    reg = torch.zeros(S, dtype=torch.int64, device=dev)
    exp = np.zeros(S, np.uint64)
    for k in range(3):
        offs = W.ragged_offsets(500 + k, S, 3000)
        payload = W.random_bytes(600 + k, int(offs[-1]) + 1)
        engine.crc64_stream_update_dev(reg, to_dev(payload, dev),
                                       to_dev(offs.view(np.int64), dev))
        exp = oracle.crc64_stream_update(exp, payload, offs)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host_np(reg).view(np.uint64), exp)


def test_stream_update_errors_and_empty(engine):
    """Error conventions (include/jrq.h): non-monotone offsets -> JRQ_E_INVALID, nothing
    written; S = 0 is a no-op; an all-empty chunk batch leaves every register unchanged
    (CRC64.update with len 0, CRC64.java:106-110)."""
    from jraft_amd._lib import JrqError
    st = np.array([5, 7], np.uint64)
    with pytest.raises(JrqError):
        engine.crc64_stream_update(st, np.zeros(16, np.uint8), np.array([0, 9, 4], np.uint64))
    assert engine.crc64_stream_update(np.zeros(0, np.uint64), np.zeros(1, np.uint8),
                                      np.array([0], np.uint64)).size == 0
    regs = np.array([0, 0x123456789ABCDEF0, 2**64 - 1], np.uint64)
    got = engine.crc64_stream_update(regs, np.zeros(4, np.uint8), np.array([2, 2, 2, 2], np.uint64))
    np.testing.assert_array_equal(got, regs)
    with pytest.raises(ValueError):
        engine.crc64_stream_update(np.zeros(3, np.uint64), np.zeros(4, np.uint8),
                                   np.array([0, 4], np.uint64))


@pytest.mark.parametrize("offs", [[0, 9, 4, 16], [5, 2, 16], [4, 9, 12, 3]])
def test_batch_offsets_must_be_monotone(engine, offs):
    """jrq_crc64_batch / jrq_logentry_checksum_batch reject offsets that go backwards (or
    below offsets[0]) with JRQ_E_INVALID before staging anything: the kernels' segment walk
    and boundary search assume sorted offsets (include/jrq.h)."""
    from jraft_amd._lib import JrqError
    offs = np.array(offs, np.uint64)
    n = len(offs) - 1
    payload = np.arange(32, dtype=np.uint8)
    with pytest.raises(JrqError, match="monotone"):
        engine.crc64_batch(payload, offs)
    with pytest.raises(JrqError, match="monotone"):
        engine.logentry_checksum_batch(np.ones(n, np.uint8), np.arange(n), np.ones(n), None,
                                       payload, offs)
    # the engine stays usable after a refused call
    ok = engine.crc64_batch(payload, np.array([0, 9, 16], np.uint64))
    assert ok.shape == (2,)

