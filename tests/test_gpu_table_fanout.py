"""GPU: the table epoch with the commit fan-out fused in (include/jrq.h jrq_table_epoch_fanout,
jrq_table_fsm_update / _read).

For every group whose commit moves in the epoch, FSMCallerImpl.doCommitted's gate and
ClosureQueueImpl.popClosureUntil on the new lastCommittedIndex (JC/core/FSMCallerImpl.java:462-482,
JC/closure/ClosureQueueImpl.java:113-142), from the FSMCaller state the table keeps beside the
BallotBox state.  Checked against the oracle: the epoch against its BallotBox replay
(BallotBox.java:96-139), the fan-out against its call-by-call doCommitted replay
(jo_commit_fanout_replay) with one onCommitted call per moved group, the queues after the pops
against the replay's.
"""
import numpy as np
import pytest

import jraft_oracle as O
from jraft_amd import JrqError, Table, decode_changed
from quorum_cases import random_batch
from test_gpu_table import committed_from, match_recs, states_of

pytestmark = pytest.mark.gpu


def fsm_state(seed, lc, committed):
    """lastAppliedIndex and ClosureQueue (firstIndex, size) per group: queues that pop, empty
    ones, ones starting past the commit, too short ones (INVALID), and applied cursors already
    past the commit (SKIP)."""
    rng = np.random.default_rng(seed)
    G = len(lc)
    kind = rng.integers(0, 5, G)
    applied = lc - rng.integers(0, 3, G)
    applied = np.where(kind == 4, committed + rng.integers(0, 5, G), applied)  # SKIP
    first = lc + 1 + np.where(kind == 2, rng.integers(1, 1000, G), 0)          # starts later
    need = np.maximum(committed - first + 1, 0)
    size = need + rng.integers(0, 50, G)
    size = np.where(kind == 1, 0, size)                                           # empty
    size = np.where(kind == 3, np.maximum(need - 1 - rng.integers(0, 3, G), 0), size)  # short
    return applied.astype(np.int64), first.astype(np.int64), size.astype(np.int64)


def oracle_fanout(lc, committed, applied, first, size):
    moved = committed > lc
    so = np.concatenate([[0], np.cumsum(moved)]).astype(np.uint64)
    st, fc, _, cf, cs, _ = O.commit_fanout_replay(so, committed[moved], applied, first, size)
    return st, fc, cf, cs


def load(engine, b, P, G):
    t = Table(engine, G, P)
    t.update(states_of(b), match_recs(b["match"], b["pending_index"]))
    return t


@pytest.mark.parametrize("P,G,runs", [(5, 20000, 0.3), (3, 3001, 0.4), (16, 777, 0.5), (1, 64, 0.0),
                                      (9, 70001, 0.1)])
def test_fused_fanout_vs_oracle(engine, oracle, P, G, runs):
    b = random_batch(4000 + P, G, P, run_prob=runs)
    ce, _, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                          b["last_committed"], b["conf"], b["run_off"],
                                          b["run_start"], b["run_conf"], chunk=7)
    lc = b["last_committed"].astype(np.int64)
    applied, first, size = fsm_state(P * 7 + G, lc, ce)
    t = load(engine, b, P, G)
    t.fsm_update(np.arange(G), applied, first, size)
    a0, f0, s0 = t.fsm_read()
    np.testing.assert_array_equal(a0, applied)
    np.testing.assert_array_equal(f0, first)
    np.testing.assert_array_equal(s0, size)
    changed, ff, fs = t.epoch_fanout()
    got, listed = committed_from(changed, b["pending_index"], lc)
    np.testing.assert_array_equal(got, ce)
    st, fc, cf, cs = oracle_fanout(lc, ce, applied, first, size)
    assert (st[listed] != O.FAN_NONE).all() and (st[np.setdiff1d(np.arange(G), listed)] == O.FAN_NONE).all()
    np.testing.assert_array_equal(fs, st[listed])
    np.testing.assert_array_equal(ff, fc[listed])
    a1, f1, s1 = t.fsm_read()
    np.testing.assert_array_equal(a1, applied)  # the host moves lastAppliedIndex after applying
    np.testing.assert_array_equal(f1, cf)
    np.testing.assert_array_equal(s1, cs)
    kinds = {int(k) for k in np.unique(fs)}
    if G >= 3000:
        assert kinds == {O.FAN_APPLY, O.FAN_SKIP, O.FAN_INVALID}, kinds
    # the plain epoch of an identically loaded table commits the same (the fused path changes
    # nothing of the BallotBox state)
    t2 = load(engine, b, P, G)
    c2, _ = t2.epoch()
    np.testing.assert_array_equal(np.sort(c2), np.sort(changed))


def test_fused_fanout_device_slices(engine, oracle):
    """The device variant's slice-shaped fan arrays, decoded in list order, equal the host
    variant's on an identically loaded table."""
    import torch

    P, G = 5, 40001
    b = random_batch(77, G, P, run_prob=0.2)
    lc = b["last_committed"].astype(np.int64)
    ce, _, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"], lc,
                                          b["conf"], b["run_off"], b["run_start"], b["run_conf"], chunk=7)
    applied, first, size = fsm_state(5, lc, ce)
    th = load(engine, b, P, G)
    th.fsm_update(np.arange(G), applied, first, size)
    ch, ffh, fsh = th.epoch_fanout()
    td = load(engine, b, P, G)
    td.fsm_update(np.arange(G), applied, first, size)
    dev = torch.device("cuda:0")
    out, nout = td.list_buffers(dev)
    ffd, fsd = td.fan_buffers(dev)
    td.epoch_fanout_dev(out, nout, ffd, fsd)
    from devio import host_np
    words = td.gather_dev_list(out, nout)
    np.testing.assert_array_equal(words, ch)
    n = host_np(nout)
    ffa, fsa = host_np(ffd), host_np(fsd)
    ff = np.concatenate([ffa[s * 128: s * 128 + n[s]] for s in range(len(n))])
    fs = np.concatenate([fsa[s * 128: s * 128 + n[s]] for s in range(len(n))])
    np.testing.assert_array_equal(ff, ffh)
    np.testing.assert_array_equal(fs, fsh)
    for x, y in zip(td.fsm_read(), th.fsm_read()):
        np.testing.assert_array_equal(x, y)


def test_fsm_update_refuses_groups_past_the_table(engine):
    t = Table(engine, 100, 3)
    t.fsm_update(np.array([5, 100, 7]), np.array([1, 2, 3]), np.array([4, 5, 6]), np.array([7, 8, 9]))
    with pytest.raises(JrqError):
        t.check()
    a, f, s = t.fsm_read()
    assert (a[5], f[5], s[5], a[7], f[7], s[7]) == (1, 4, 7, 3, 6, 9)
