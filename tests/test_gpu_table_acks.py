"""GPU: order-free ack records (include/jrq.h JRQ_ACK, jrq_table_stage_acks).

What BallotBox.commitAt / appendPendingTask record at call time (the absolute index's low 32
bits) is applied by the device as an order-free max after the headers of the same update; a
record stamped before its group's last reset (JRQ_STATE_STAMP header) is dropped.  Every epoch
is checked against the oracle's BallotBox replay (BallotBox.java:96-139) on the matches the
records amount to.
"""
import numpy as np
import pytest

from jraft_amd import JrqError, Table, _lib, decode_changed
from jraft_amd import conf_word

pytestmark = pytest.mark.gpu


def _headers(G, pi, la, lc, cw, flags=_lib.STATE_RESET_MATCH, stamp=None):
    st = Table.states(G)
    st["group"] = np.arange(G)
    st["num_runs"] = 1
    st["flags"] = flags | (_lib.STATE_STAMP if stamp is not None else 0)
    st["pending_index"] = pi
    st["last_appended"] = la
    st["last_committed"] = lc
    st["run_conf"][:, 0] = cw
    if stamp is not None:
        st["run_start"][:, 0] = stamp
    return st


def _committed(changed, pi, lc):
    g, d = decode_changed(changed)
    out = lc.copy()
    out[g] = pi[g] - 1 + d
    return out


@pytest.mark.parametrize("base", [1 << 20, (1 << 32) - 700, (1 << 31) - 300, 7 << 30])
def test_acks_order_free_max_vs_replay(engine, oracle, base):
    """Shuffled records with duplicates and stale (lower) values, in three segments: the epoch
    equals the replay on the per-slot maxima; windows straddling 2^31, 2^32 and match-base
    boundaries reconstruct from the low 32 bits."""
    rng = np.random.default_rng(base & 0xFFFF)
    G, P = 3000, 5
    pi = base + rng.integers(0, 500, G)
    lc = pi - 1
    la0 = pi + 200
    cw = np.full(G, conf_word(0b11111, 0b00111), np.uint64)
    t = Table(engine, G, P)
    try:
        t.update(_headers(G, pi, la0, lc, cw))
        la = la0 + rng.integers(0, 600, G)          # appends recorded as la records (max)
        m = (pi - 1)[None, :] + rng.integers(0, 800, (P, G))
        m = np.minimum(m, la[None, :])
        recs = [_lib.ack(np.arange(G), _lib.REC_LAST_APPENDED, la)]
        recs.append(_lib.ack(np.arange(G), _lib.REC_LAST_APPENDED, la0))  # stale, lower
        for p in range(P):
            recs.append(_lib.ack(np.arange(G), p, m[p]))
            recs.append(_lib.ack(np.arange(G), p, m[p] - rng.integers(0, 50, G)))  # older acks
        allr = np.concatenate(recs)
        rng.shuffle(allr)
        t.stage_reserve(0, 0, len(allr), 4)
        k = len(allr) // 3
        t.stage_acks(0, allr[:k])
        t.stage_acks(0, allr[k:2 * k])
        t.stage_acks(0, allr[2 * k:])
        t.stage_apply()
        ce, se, _ = oracle.quorum_epoch_replay(m, pi, la, lc, cw, chunk=64)
        changed, st = t.epoch(status=True)
        np.testing.assert_array_equal(_committed(changed, pi, lc), ce)
        np.testing.assert_array_equal(st, se)
        r = t.read()
        np.testing.assert_array_equal(r["last_appended"], la)
        t.check()
    finally:
        t.close()


def test_acks_dropped_before_reset_stamp(engine, oracle):
    """Records stamped before a group's reset (a header with JRQ_STATE_STAMP) are dropped; the
    ones stamped at or after it apply.  A non-leader group ignores records."""
    G, P = 512, 3
    pi = np.full(G, 1000, np.int64)
    lc = pi - 1
    la = pi + 100
    cw = np.full(G, conf_word(0b111), np.uint64)
    t = Table(engine, G, P)
    try:
        old = np.arange(G) % 2 == 0          # even groups: reset (stamp 7) after their old acks
        t.update(_headers(G, pi, la, lc, cw, stamp=np.where(old, 7, 0)))
        m_old = np.where(old, pi + 80, pi + 10)   # acks at stamp 6: dropped for even groups
        m_new = pi + 40                           # acks at stamp 7: applied everywhere
        recs6 = np.concatenate([_lib.ack(np.arange(G), p, m_old) for p in range(P)])
        recs7 = np.concatenate([_lib.ack(np.arange(G), p, m_new) for p in range(P)])
        # group 5 is not the leader: its records are ignored
        st5 = _headers(1, 0, -1, 3, 0, flags=0)
        st5["group"] = 5
        st5["num_runs"] = 0
        t.update(st5)
        t.stage_reserve(0, 0, len(recs6) + len(recs7), 2)
        t.stage_acks(6, recs6)
        t.stage_acks(7, recs7)
        t.stage_apply()
        m = np.where(old, m_new, np.maximum(m_old, m_new))
        mm = np.broadcast_to(m, (P, G)).copy()
        pi2, lc2, la2 = pi.copy(), lc.copy(), la.copy()
        pi2[5], lc2[5], la2[5] = 0, 3, -1
        ce, _, _ = oracle.quorum_epoch_replay(mm, pi2, la2, lc2, np.where(np.arange(G) == 5, 0, cw).astype(np.uint64), chunk=64)
        changed, _ = t.epoch()
        np.testing.assert_array_equal(_committed(changed, pi2, lc2), ce)
        assert ce[0] == 1000 + 40 and ce[1] == 1000 + 40 and ce[5] == 3
        t.check()
    finally:
        t.close()


def test_invalid_ack_records_counted(engine):
    G, P = 64, 3
    pi = np.full(G, 10, np.int64)
    t = Table(engine, G, P)
    try:
        t.update(_headers(G, pi, pi + 5, pi - 1, np.full(G, conf_word(0b111), np.uint64)))
        bad = np.array([_lib.ack(G + 3, 0, 12), _lib.ack(1, 7, 12), _lib.ack(1, 17, 12),
                        _lib.ack(2, _lib.REC_LAST_APPENDED, 10 + (1 << 31))], np.uint64)
        t.stage_reserve(0, 0, len(bad), 1)
        t.stage_acks(0, bad)
        t.stage_apply()
        t.epoch()
        with pytest.raises(JrqError):
            t.check()
        assert t.read()["last_appended"][2] == 15
    finally:
        t.close()
