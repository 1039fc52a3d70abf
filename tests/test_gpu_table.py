"""GPU parity of the resident group table (include/jrq.h jrq_table, csrc/table.hip) against the
oracle's Java-faithful BallotBox replays (jraft-core/.../core/BallotBox.java:96-248).

The table is loaded the way a host drives it: group headers for resetPendingIndex / conf runs,
8-byte records for commitAt acks and appendPendingTask queue growth (values relative to the
group's pendingIndex), then epochs that return only the groups whose commit advanced.
"""
import numpy as np
import pytest

from jraft_amd import JrqError, Table, decode_changed
from jraft_amd import _lib
from quorum_cases import random_batch, random_series, series_replay
from devio import to_dev, host_np

pytestmark = pytest.mark.gpu


def states_of(b, groups=None):
    """jrq_group_state records of a random_batch / random_series dict (runs from its CSR)."""
    G = len(b["pending_index"])
    groups = np.arange(G) if groups is None else groups
    st = Table.states(len(groups))
    ro = b["run_off"]
    for i, g in enumerate(groups):
        r0, r1 = int(ro[g]), int(ro[g + 1])
        st[i]["group"] = g
        st[i]["num_runs"] = r1 - r0
        st[i]["flags"] = _lib.STATE_RESET_MATCH
        st[i]["pending_index"] = b["pending_index"][g]
        la = b["last_appended"]
        st[i]["last_appended"] = la[g] if la.ndim == 1 else la[0][g]
        st[i]["last_committed"] = b["last_committed"][g]
        st[i]["run_conf"][: r1 - r0] = b["run_conf"][r0:r1]
        st[i]["run_start"][: r1 - r0] = b["run_start"][r0:r1]
    return st


def match_recs(match, pi, groups=None):
    """Records setting every slot's match (relative to pendingIndex; below it = 0)."""
    P, G = match.shape
    gs = np.arange(G) if groups is None else np.asarray(groups)
    lead = pi[gs] != 0
    gs = gs[lead]
    out = []
    for p in range(P):
        v = np.maximum(match[p, gs] - (pi[gs] - 1), 0)
        out.append(_lib.rec(gs, p, v))
    return np.concatenate(out) if out else np.zeros(0, np.uint64)


def la_recs(la, pi, groups):
    gs = np.asarray(groups)
    gs = gs[pi[gs] != 0]
    return _lib.rec(gs, _lib.REC_LAST_APPENDED, la[gs] - (pi[gs] - 1))


def committed_from(changed, pi_before, lc_before):
    g, d = decode_changed(changed)
    out = lc_before.copy()
    assert len(np.unique(g)) == len(g), "a group listed twice"
    out[g] = pi_before[g] - 1 + d
    return out, g


@pytest.mark.parametrize("P,G,runs", [(5, 4096, 0.4), (3, 3001, 0.4), (16, 777, 0.4), (1, 64, 0.4),
                                      (5, 70001, 0.95), (9, 20001, 0.4), (16, 9000, 0.9)])
def test_one_epoch_vs_replay(engine, oracle, P, G, runs):
    """One epoch vs the BallotBox replay.  The last case has 35 workgroups (several per list
    segment, a pad group) and nearly every group walking conf runs (many quad-walk passes
    per workgroup)."""
    b = random_batch(1000 + P, G, P, run_prob=runs)
    ce, se, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                           b["last_committed"], b["conf"], b["run_off"],
                                           b["run_start"], b["run_conf"], chunk=7)
    t = Table(engine, G, P)
    t.update(states_of(b), match_recs(b["match"], b["pending_index"]))
    changed, st = t.epoch(status=True)
    got, listed = committed_from(changed, b["pending_index"], b["last_committed"])
    np.testing.assert_array_equal(got, ce)
    np.testing.assert_array_equal(np.sort(listed), np.nonzero(ce > b["last_committed"])[0])
    np.testing.assert_array_equal(st, se)
    # the state moved as BallotBox moves it (pendingIndex = commit + 1, read through the
    # JRQ_PI_FOLLOWS_LC word), and a second epoch with no new acks commits nothing
    r = t.read()
    np.testing.assert_array_equal(r["last_committed"], ce)
    moved = ce > b["last_committed"]
    np.testing.assert_array_equal(r["pending_index"][moved], ce[moved] + 1)
    np.testing.assert_array_equal(r["pending_index"][~moved], b["pending_index"][~moved])
    again, _ = t.epoch()
    assert len(again) == 0
    t.close()


@pytest.mark.parametrize("P,G,K", [(3, 2000, 6), (5, 1500, 5)])
def test_epochs_incremental_vs_replays(engine, oracle, P, G, K):
    """K epochs driven incrementally -- per epoch only the queue sizes and the acks that
    changed -- equal K sequential BallotBox replays with carried state."""
    s = random_series(77 + P, G, P, K)
    ce, se = series_replay(oracle, s)
    t = Table(engine, G, P)
    pi = s["pending_index"].copy()
    lc = s["last_committed"].copy()
    t.update(states_of(s), match_recs(s["match"][0], pi))
    for k in range(K):
        if k > 0:
            la_changed = np.nonzero(s["last_appended"][k] != s["last_appended"][k - 1])[0]
            recs = [la_recs(s["last_appended"][k], pi, la_changed)]
            for p in range(P):
                ch = np.nonzero(s["match"][k, p] != s["match"][k - 1, p])[0]
                ch = ch[pi[ch] != 0]
                recs.append(_lib.rec(ch, p, np.maximum(s["match"][k, p, ch] - (pi[ch] - 1), 0)))
            t.update(None, np.concatenate(recs))
        changed, st = t.epoch(status=True)
        got, listed = committed_from(changed, pi, lc)
        np.testing.assert_array_equal(got, ce[k], err_msg=f"epoch {k}")
        np.testing.assert_array_equal(st, se[k], err_msg=f"epoch {k}")
        pi[listed] = got[listed] + 1
        lc = got
    t.close()


def test_group_state_resets_and_clears(engine, oracle):
    """resetPendingIndex with RESET_MATCH wipes old acks; clearPendingTasks (pendingIndex 0)
    stops commits; records are relative to the pendingIndex the headers just set."""
    from jraft_amd import conf_word
    G = 256
    b = random_batch(5, G, 3, run_prob=0.0, edge=False)
    t = Table(engine, G, 3)
    t.update(states_of(b), match_recs(b["match"], b["pending_index"]))
    t.epoch()
    st = states_of(b)
    st["pending_index"] = b["pending_index"] + 5000
    st["last_appended"] = st["pending_index"] + 9  # 10 entries pending
    st["last_committed"] = b["pending_index"] + 4000
    st["num_runs"] = 1
    st["run_conf"][:, 0] = conf_word(0b111)
    t.update(st)
    changed, _ = t.epoch()
    assert len(changed) == 0  # every match was reset below the new pendingIndex
    clr = states_of(b, groups=[0, 1])
    clr["pending_index"] = 0
    clr["num_runs"] = 0
    gs = np.arange(G)
    t.update(clr, np.concatenate([_lib.rec(gs[2:], 0, 10), _lib.rec(gs[2:], 1, 7)]))
    changed, stt = t.epoch(status=True)
    g, d = decode_changed(changed)
    assert sorted(g.tolist()) == list(range(2, G))
    assert (d == 7).all()  # quorum 2 of 3: the 7th pending entry
    assert (stt[:2] == _lib.ST_NOT_LEADER).all()
    r = t.read()
    np.testing.assert_array_equal(r["last_committed"][2:], st["pending_index"][2:] + 6)
    t.close()


def test_invalid_records_skipped_and_reported(engine):
    """Out-of-range headers / records never touch the table: the kernels skip and count them,
    jrq_table_check reports them once."""
    t = Table(engine, 100, 3)
    t.check()
    for bad in (_lib.rec(100, 0, 1), _lib.rec(5, 3, 1), _lib.rec(5, 17, 1)):
        t.update(None, np.atleast_1d(bad))
        with pytest.raises(JrqError):
            t.check()
        t.check()  # reported once, then reset
    st = Table.states(2)
    st["group"] = [100, 1]
    st["num_runs"] = [1, 5]
    t.update(st)
    with pytest.raises(JrqError, match="2 group headers"):
        t.check()
    r = t.read()
    assert (r["pending_index"] == 0).all() and (r["match"] == 0).all()
    t.close()


def test_device_variant_and_view(engine, oracle):
    """The _dev entry points on torch buffers, and the view's lastCommitted row (the rank's
    all-gather send buffer)."""
    import torch
    G, P = 2048, 5
    b = random_batch(9, G, P, run_prob=0.1)
    ce, _, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                          b["last_committed"], b["conf"], b["run_off"],
                                          b["run_start"], b["run_conf"], chunk=3)
    t = Table(engine, G, P)
    dev = torch.device("cuda:0")
    st = to_dev(states_of(b).view(np.uint8), dev)
    rc = to_dev(match_recs(b["match"], b["pending_index"]).view(np.int64), dev)
    t.update_dev(st, rc)
    out, n = t.list_buffers(dev)
    t.epoch_dev(out, n)
    engine.synchronize()
    got, _ = committed_from(t.gather_dev_list(out, n), b["pending_index"], b["last_committed"])
    np.testing.assert_array_equal(got, ce)
    v = t.view()
    assert v.G == G and v.num_peers == P and v.ld >= G and v.last_committed
    assert v.tile_groups == 256 and v.tile_stride == 128 * P + 1024
    # lastCommitted of group g through the view's tiled addressing, and the u32 match words
    lcd = torch.empty(((G + 255) // 256) * v.tile_stride, dtype=torch.int64, device=dev)
    import ctypes  # (the view holds raw device pointers: read the tiles through hipMemcpy)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(lcd.data_ptr()), ctypes.c_void_p(v.match), lcd.numel() * 8, 3) == 0
    words = host_np(lcd)
    g = np.arange(G)
    assert v.last_committed == v.match + 8 * (128 * P + 512)
    lc_view = words[(g // 256) * v.tile_stride + 128 * P + 512 + g % 256]
    np.testing.assert_array_equal(lc_view, ce)
    rd = t.read()
    np.testing.assert_array_equal(rd["last_committed"], ce)
    k = g % 256
    pos = k  # the view's documented order: group order within the tile
    u32 = words.view(np.uint32)
    pi = rd["pending_index"]
    base = np.where(pi > 0, (pi - 1) & ~np.int64((1 << 30) - 1), 0)
    for p in range(P):
        w = u32[(g // 256) * 2 * v.tile_stride + 256 * p + pos].astype(np.int64)
        np.testing.assert_array_equal(base + w, rd["match"][p])
    # every leader's match at or above pendingIndex - 1 reads back exactly (below: raised to
    # the base; match_recs sends none for non-leaders)
    m = b["match"]
    exact = (m >= (pi - 1)[None, :]) & (pi > 0)[None, :]
    np.testing.assert_array_equal(rd["match"][exact], m[exact])
    t.close()


def test_reset_header_in_follows_lc_encoding(engine):
    """A new leader's header in the steady-state encoding (pendingIndex = lastCommitted + 1 sent
    as JRQ_PI_FOLLOWS_LC, as GroupBatch::flush sends it after setLastCommittedIndex +
    resetPendingIndex(lc + 1)) with RESET_MATCH: every slot's match becomes pendingIndex - 1,
    nothing reports OUT_OF_RANGE, and later acks commit as usual."""
    from jraft_amd import conf_word
    G, P = 130, 3
    t = Table(engine, G, P)
    st = Table.states(G)
    st["group"] = np.arange(G)
    st["num_runs"] = 1
    st["flags"] = _lib.STATE_RESET_MATCH
    lc = 1000 + np.arange(G, dtype=np.int64) * 7
    st["pending_index"] = _lib.PI_FOLLOWS_LC
    st["last_committed"] = lc
    st["last_appended"] = lc + 10
    st["run_conf"][:, 0] = conf_word(0b111)
    t.update(st)
    r = t.read()
    np.testing.assert_array_equal(r["pending_index"], lc + 1)
    np.testing.assert_array_equal(r["match"], np.broadcast_to(lc, (P, G)))
    changed, stt = t.epoch(status=True)
    assert len(changed) == 0 and (stt == 0).all()
    gs = np.arange(G)
    t.update(None, np.concatenate([_lib.rec(gs, 0, 4), _lib.rec(gs, 2, 6)]))
    changed, stt = t.epoch(status=True)
    g, d = decode_changed(changed)
    assert sorted(g.tolist()) == list(range(G)) and (d == 4).all() and (stt == 0).all()
    t.check()
    t.close()


def test_pending_entries_without_conf_run_are_invalid(engine):
    """A leader header with entries pending but no conf run (conf word 0 = quorum 0, which would
    grant everything), or a queue-size record growing such a group's queue, is refused and
    reported; the group then commits nothing whatever it is acked."""
    t = Table(engine, 8, 3)
    st = Table.states(1)
    st["group"] = 2
    st["num_runs"] = 0
    st["pending_index"] = 10
    st["last_committed"] = 9
    st["last_appended"] = 12
    t.update(st)
    with pytest.raises(JrqError):
        t.check()
    st["last_appended"] = 9   # nothing pending (what resetPendingIndex leaves): valid
    t.update(st)
    t.check()
    t.update(None, np.atleast_1d(_lib.rec(2, _lib.REC_LAST_APPENDED, 3)))
    with pytest.raises(JrqError):
        t.check()
    t.update(None, np.concatenate([np.atleast_1d(_lib.rec(2, p, 3)) for p in range(3)]))
    changed, _ = t.epoch()
    assert len(changed) == 0
    assert t.read()["last_appended"][2] == 9
    t.check()
    t.close()


@pytest.mark.parametrize("G,joint", [(20000, 0.05), (4097, 0.9), (70000, 0.0)])
def test_flagged_groups_in_full_blocks(engine, G, joint):
    """Every group commits (C3 host series) and some have a conf change in their window: a
    workgroup lists its own groups only -- committing single-conf ones and walked flagged ones --
    so no list segment overflows; against the stateless kernel with the CSR run table, through
    both the host variant and the _dev segments, twice (the flagged lists after reloads)."""
    import torch

    from jraft_amd import workloads as W
    s = W.host_series("C3", 1, groups=G, joint_frac=joint)
    P = 5
    pi = s["pending_index"]
    st = Table.states(G)
    jm = s["switch_at"] != 0
    st["group"] = np.arange(G)
    st["num_runs"] = np.where(jm, 2, 1)
    st["flags"] = _lib.STATE_RESET_MATCH
    st["pending_index"] = np.where(pi == s["last_committed"] + 1, _lib.PI_FOLLOWS_LC, pi)
    st["last_appended"] = s["last_appended"][0]
    st["last_committed"] = s["last_committed"]
    st["run_conf"][:, 0] = s["conf_a"]
    st["run_conf"][:, 1] = np.where(jm, s["conf_b"], 0)
    st["run_start"][:, 1] = s["switch_at"]
    m = s["match"][0]
    gs = np.arange(G)
    recs = np.concatenate([_lib.rec(gs, p, np.maximum(m[p] - (pi - 1), 0)) for p in range(P)])
    dev = torch.device("cuda:0")
    d = {k: to_dev(np.ascontiguousarray(v.view(np.int64) if v.dtype == np.uint64 else v), dev)
         for k, v in (("match", m), ("pi", pi), ("la", s["last_appended"][0]),
                      ("lc", s["last_committed"]), ("conf", s["conf"]), ("run_off", s["run_off"]),
                      ("run_start", s["run_start"]), ("run_conf", s["run_conf"]))}
    pc = torch.empty(G, dtype=torch.int64, device=dev)
    ps = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_dev(d["match"], d["pi"], d["la"], d["lc"], d["conf"], pc, ps,
                            run_off=d["run_off"], run_start=d["run_start"], run_conf=d["run_conf"])
    engine.synchronize()
    exp_c, exp_s = host_np(pc), host_np(ps)
    assert (exp_c > s["last_committed"]).mean() > 0.9
    t = Table(engine, G, P)
    for rep in range(2):
        t.update(st, recs)
        if rep == 0:
            changed, stt = t.epoch(status=True)
        else:
            out, n = t.list_buffers(dev)
            sd = torch.empty(G, dtype=torch.uint8, device=dev)
            t.epoch_dev(out, n, sd)
            engine.synchronize()
            assert (host_np(n) <= _lib.TABLE_SLICE).all()
            changed, stt = t.gather_dev_list(out, n), host_np(sd)
        got, _ = committed_from(changed, pi, s["last_committed"])
        np.testing.assert_array_equal(got, exp_c)
        np.testing.assert_array_equal(stt, exp_s)
    t.check()
    t.close()


@pytest.mark.parametrize("G", [64, 300, 1000])
def test_epoch_dev_writes_only_its_slices(engine, G):
    """The epoch grid is whole workgroups (4 waves of 256 groups): a wave past the last slice
    owns no slice and must write nothing -- the caller's list holds jrq_table_slices(t) slices
    and its counts exactly that many words.  Sentinels after both buffers stay intact."""
    import torch
    P = 3
    b = random_batch(77, G, P, run_prob=0.2)
    t = Table(engine, G, P)
    t.update(states_of(b), match_recs(b["match"], b["pending_index"]))
    dev = torch.device("cuda:0")
    S = t.slices()
    pad = 4 * _lib.TABLE_SLICE
    out = torch.full((S * _lib.TABLE_SLICE + pad,), -7, dtype=torch.int64, device=dev)
    n = torch.full((S + 64,), -7, dtype=torch.int32, device=dev)
    st = torch.full((G + 64,), 0xEE, dtype=torch.uint8, device=dev)
    t.epoch_dev(out[:S * _lib.TABLE_SLICE], n[:S], st[:G])
    engine.synchronize()
    assert (out[S * _lib.TABLE_SLICE:] == -7).all().item()
    assert (n[S:] == -7).all().item()
    assert (st[G:] == 0xEE).all().item()
    t.close()


@pytest.mark.parametrize("P,joint", [(3, False), (5, True)])
def test_match_base_rebase_across_2_30(engine, oracle, P, joint):
    """The v3 layout keeps match as u32 words against mbase(pi) = (pi - 1) & ~(2^30 - 1).  Groups
    whose commit carries pendingIndex across a 2^30 boundary (near 2^30 and near 2^31) have their
    words rebased by the committing wave; the next epoch's acks (relative to the new
    pendingIndex) must decide exactly as two carried BallotBox replays, and jrq_table_read must
    return the absolute match of every slot at or above the new base."""
    from jraft_amd import conf_word
    G = 600
    rng = np.random.default_rng(31 + P)
    g = np.arange(G)
    base0 = np.where(g % 2 == 0, 1 << 30, 1 << 31).astype(np.int64)
    pi = base0 - 150 + (g % 200)                     # some cross the boundary, some do not
    lc = pi - 1
    la = pi + 500
    cw = conf_word((1 << P) - 1, 0b111 if joint else 0)
    conf = np.full(G, cw, np.uint64)
    st = Table.states(G)
    st["group"] = g
    st["num_runs"] = 1
    st["flags"] = _lib.STATE_RESET_MATCH
    st["pending_index"] = pi
    st["last_appended"] = la
    st["last_committed"] = lc
    st["run_conf"][:, 0] = cw
    t = Table(engine, G, P)
    t.update(st)
    m1 = (pi - 1)[None, :] + rng.integers(0, 320, (P, G))
    m1 = np.minimum(m1, la[None, :])
    t.update(None, match_recs(m1, pi))
    ce1, se1, _ = oracle.quorum_epoch_replay(m1, pi, la, lc, conf, chunk=64)
    changed, st1 = t.epoch(status=True)
    got1, listed = committed_from(changed, pi, lc)
    np.testing.assert_array_equal(got1, ce1)
    np.testing.assert_array_equal(st1, se1)
    crossed = ((pi - 1) >> 30) != ((np.where(ce1 > lc, ce1 + 1, pi) - 1) >> 30)
    assert crossed.sum() > 50 and (~crossed).sum() > 50  # both kinds present
    pi1 = np.where(ce1 > lc, ce1 + 1, pi)
    r = t.read()
    np.testing.assert_array_equal(r["pending_index"], pi1)
    nb = (pi1 - 1) & ~np.int64((1 << 30) - 1)
    keep = m1 >= nb[None, :]
    np.testing.assert_array_equal(r["match"][keep], m1[keep])
    np.testing.assert_array_equal(r["match"][~keep], np.broadcast_to(nb, (P, G))[~keep])
    # epoch 2: the queue grows and new acks arrive, relative to the new pendingIndex
    la2 = pi1 + 400
    m2 = np.maximum(m1, (pi1 - 1)[None, :] + rng.integers(0, 380, (P, G)))
    m2 = np.minimum(m2, la2[None, :])
    recs = [la_recs(la2, pi1, g)]
    for p in range(P):
        ch = np.nonzero(m2[p] != m1[p])[0]
        recs.append(_lib.rec(ch, p, np.maximum(m2[p, ch] - (pi1[ch] - 1), 0)))
    t.update(None, np.concatenate(recs))
    ce2, se2, _ = oracle.quorum_epoch_replay(m2, pi1, la2, ce1, conf, chunk=64)
    changed, st2 = t.epoch(status=True)
    got2, _ = committed_from(changed, pi1, ce1)
    np.testing.assert_array_equal(got2, ce2)
    np.testing.assert_array_equal(st2, se2)
    t.check()
    t.close()


def test_lowered_base_without_reset_invents_no_ack(engine):
    """a header without RESET_MATCH that lowers a leader's match base.
    Slots whose word is 0 under the old base (match at or below it: unknown) must not read back
    as exactly the old base -- that would count as an ack of entries no peer acknowledged.
    Such words stay 0 (no grant); words above 0 are shifted exactly."""
    from jraft_amd import conf_word
    G, P = 4, 3
    B = 1 << 30
    cw = conf_word(0b111, 0)
    st = Table.states(G)
    st["group"] = np.arange(G)
    st["num_runs"] = 1
    st["flags"] = _lib.STATE_RESET_MATCH
    st["pending_index"] = B + 1          # base B: every slot's word 0 (match = B)
    st["last_appended"] = B + 40
    st["last_committed"] = B
    st["run_conf"][:, 0] = cw
    t = Table(engine, G, P)
    t.update(st)
    # slot 0 of every group acks B + 5 (word 5); slots 1, 2 stay at word 0
    t.update(None, _lib.rec(np.arange(G), 0, np.full(G, 5)))  # match = pi - 1 + 5 = B + 5
    # the non-reset header: pendingIndex lowered below the base (base 0 afterwards)
    st2 = st.copy()
    st2["flags"] = 0
    st2["pending_index"] = B - 10
    st2["last_committed"] = B - 11
    st2["last_appended"] = B + 40
    t.update(st2)
    r = t.read()
    np.testing.assert_array_equal(r["match"][0], np.full(G, B + 5))   # shifted exactly
    np.testing.assert_array_equal(r["match"][1:], 0)                  # unknown: no ack
    changed, _ = t.epoch(status=True)
    assert len(changed) == 0  # quorum 2 of 3: one real ack (slot 0) is not a quorum
    # a real ack of slot 1 afterwards decides normally: min(B + 5, B + 2) = B + 2
    pi2 = np.full(G, B - 10, np.int64)
    t.update(None, _lib.rec(np.arange(G), 1, np.full(G, (B + 2) - (B - 11))))
    changed, _ = t.epoch(status=True)
    got, _ = committed_from(changed, pi2, np.full(G, B - 11, np.int64))
    np.testing.assert_array_equal(got, np.full(G, B + 2))
    t.check()
    t.close()


def test_header_with_lastappended_below_pending_refused(engine):
    """lastAppended < pendingIndex - 1 is a queue of negative size, which no
    BallotBox holds; such a header is skipped and reported (the epoch's u32 out-of-range test
    relies on lastAppended >= the match base)."""
    from jraft_amd import conf_word
    G, P = 2, 3
    st = Table.states(G)
    st["group"] = np.arange(G)
    st["num_runs"] = 1
    st["flags"] = _lib.STATE_RESET_MATCH
    st["pending_index"] = [(1 << 30) + 3, 100]
    st["last_appended"] = [(1 << 30) - 7, 99]   # group 0: la < pi - 1 across the 2^30 base
    st["last_committed"] = [(1 << 30) + 2, 99]
    st["run_conf"][:, 0] = conf_word(0b111, 0)
    t = Table(engine, G, P)
    t.update(st)
    with pytest.raises(JrqError):
        t.check()
    r = t.read()
    assert r["pending_index"][0] == 0 and r["pending_index"][1] == 100  # group 0 untouched
    t.check()
    t.close()
