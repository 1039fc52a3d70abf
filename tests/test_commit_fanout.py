"""Commit fan-out after a quorum epoch: FSMCallerImpl.doCommitted ->
ClosureQueueImpl.popClosureUntil per group (JC/core/FSMCallerImpl.java:462-482,
JC/closure/ClosureQueueImpl.java:113-142).

CPU tests pin the oracle's ClosureQueue to the reference's own ClosureQueueTest and check the
engine's closed form (one evaluation on the epoch's final committed index) against the
oracle's call-by-call replay.  GPU tests run jrq_commit_fanout[_dev] against the oracle.
"""
import numpy as np
import pytest

import jraft_oracle as O
from devio import to_dev, host_np

I64_MIN = np.iinfo(np.int64).min


def closed_form(prev, committed, last_applied, cq_first, cq_size):
    """The engine's formulation (commit_fanout.hip) in numpy."""
    prev, c, la = (np.asarray(x, np.int64) for x in (prev, committed, last_applied))
    f, n = np.asarray(cq_first, np.int64).copy(), np.asarray(cq_size, np.int64).copy()
    G = len(c)
    st = np.zeros(G, np.uint8)
    fc = np.zeros(G, np.int64)
    adv = c > prev
    skip = adv & (la >= c)
    act = adv & ~skip
    empty = act & ((n == 0) | (c < f))
    invalid = act & ~empty & (c > f + n - 1)
    pop = act & ~empty & ~invalid
    st[skip] = O.FAN_SKIP
    st[empty | pop] = O.FAN_APPLY
    st[invalid] = O.FAN_INVALID
    fc[empty] = c[empty] + 1
    fc[invalid] = -1
    fc[pop] = f[pop]
    n[pop] -= c[pop] - f[pop] + 1
    f[pop] = c[pop] + 1
    return st, fc, f, n


def random_epoch(seed, G, invalid_frac=0.05):
    """Groups with a closure queue, an apply cursor and an increasing onCommitted sequence."""
    rng = np.random.default_rng(seed)
    prev = rng.integers(0, 1 << 40, G).astype(np.int64)
    qlen = rng.integers(0, 2048, G).astype(np.int64)
    # leader: closures for [prev+1 .. prev+qlen] (or a later first index), follower: empty
    kind = rng.integers(0, 4, G)
    cq_first = np.where(kind == 3, prev + 1 + rng.integers(0, 50, G), prev + 1)
    cq_size = np.where(kind == 2, 0, qlen)
    la = prev - rng.integers(0, 4, G)
    la = np.where(rng.random(G) < 0.05, prev + 5000, la)  # applied ahead (skip)
    adv = rng.integers(0, 1500, G)
    adv[rng.random(G) < 0.2] = 0  # no commit this epoch
    committed = prev + adv
    # a consistent leader queue holds a closure for every index up to lastAppended >= committed
    need = np.maximum(committed - cq_first + 1, 0)
    cq_size = np.where(kind == 2, 0, np.maximum(cq_size, need + rng.integers(0, 64, G)))
    # commit beyond the queue: only reachable from an inconsistent state, and then the engine
    # reports INVALID with nothing popped; it is tested with one onCommitted call per epoch
    # (the reference could have popped a prefix through an earlier call of the same epoch)
    bad = rng.random(G) < invalid_frac
    committed[bad] = cq_first[bad] + cq_size[bad] + rng.integers(0, 9, bad.sum())
    seqs = []
    for g in range(G):
        if committed[g] <= prev[g]:
            seqs.append([])
        elif bad[g]:
            seqs.append([int(committed[g])])  # one call: a -1 pop leaves nothing popped
        else:
            k = int(rng.integers(1, 5))
            mids = sorted(set(rng.integers(prev[g] + 1, committed[g] + 1, k - 1).tolist()))
            seqs.append([m for m in mids if m < committed[g]] + [int(committed[g])])
    seq_off = np.zeros(G + 1, np.uint64)
    seq_off[1:] = np.cumsum([len(s) for s in seqs])
    seq = np.array([x for s in seqs for x in s] or [0], np.int64)
    return dict(prev=prev, committed=committed, last_applied=la, cq_first=cq_first.astype(np.int64),
                cq_size=cq_size.astype(np.int64), seq_off=seq_off, seq=seq)


def oracle_epoch(ep):
    st, fc, la, cf, cs, _ = O.commit_fanout_replay(ep["seq_off"], ep["seq"], ep["last_applied"],
                                                   ep["cq_first"], ep["cq_size"])
    listed = np.nonzero((st == O.FAN_APPLY) | (st == O.FAN_INVALID))[0].astype(np.uint32)
    return st, fc, la, cf, cs, listed


class ClosureQueue:
    """Single popClosureUntil calls driven through the oracle (one-call epochs)."""

    def __init__(self):
        self.first, self.size = 0, 0

    def append(self, k):
        self.size += k

    def pop_until(self, end):
        st, fc, _, cf, cs, _ = O.commit_fanout_replay([0, 1], [end], [I64_MIN],
                                                      [self.first], [self.size])
        assert st[0] in (O.FAN_APPLY, O.FAN_INVALID)
        popped = self.size - int(cs[0])
        self.first, self.size = int(cf[0]), int(cs[0])
        return int(fc[0]), popped


def test_closure_queue_append_pop():
    """ClosureQueueTest.testAppendPop (JT/closure/ClosureQueueTest.java:48-91) restated."""
    q = ClosureQueue()
    q.append(10)
    assert q.first == 0
    assert q.pop_until(4) == (0, 5) and q.first == 5
    assert q.pop_until(4) == (5, 0)
    assert q.pop_until(3) == (4, 0)
    assert q.pop_until(10) == (-1, 0)
    assert q.pop_until(9) == (5, 5) and q.first == 10
    assert q.pop_until(1) == (2, 0)
    assert q.pop_until(3) == (4, 0)
    q.append(10)
    assert q.pop_until(15) == (10, 6) and q.first == 16
    assert q.pop_until(20) == (-1, 0)
    assert q.pop_until(19) == (16, 4) and q.first == 20


def test_closure_queue_reset_first_index():
    """ClosureQueueTest.testResetFirstIndex (:93-112) restated."""
    q = ClosureQueue()
    q.first = 10  # resetFirstIndex(10)
    q.append(10)
    assert q.pop_until(4) == (5, 0)
    assert q.pop_until(3) == (4, 0)
    assert q.pop_until(19) == (10, 10) and q.first == 20
    assert q.pop_until(20) == (21, 0)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_closed_form_matches_call_by_call_replay(seed):
    ep = random_epoch(seed, 3000)
    st, fc, la, cf, cs, _ = oracle_epoch(ep)
    st2, fc2, cf2, cs2 = closed_form(ep["prev"], ep["committed"], ep["last_applied"],
                                     ep["cq_first"], ep["cq_size"])
    assert np.array_equal(st, st2)
    assert np.array_equal(fc, fc2)
    assert np.array_equal(cf, cf2)
    assert np.array_equal(cs, cs2)
    applied = st == O.FAN_APPLY
    assert np.array_equal(la[applied], ep["committed"][applied])
    assert set(np.unique(st)) == {O.FAN_NONE, O.FAN_APPLY, O.FAN_SKIP, O.FAN_INVALID}


# ------------------------------------------------------------------ GPU --

@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 2, 66, 4095, 4096, 4097, 4098, 50_000])
def test_gpu_fanout_vs_oracle(engine, G):
    ep = random_epoch(100 + G, G)
    st, fc, la, cf, cs, listed = oracle_epoch(ep)
    gst, gfc, glisted, gcf, gcs = engine.commit_fanout(ep["prev"], ep["committed"],
                                                       ep["last_applied"], ep["cq_first"],
                                                       ep["cq_size"])
    assert np.array_equal(gst, st)
    assert np.array_equal(gfc, fc)
    assert np.array_equal(gcf, cf)
    assert np.array_equal(gcs, cs)
    assert np.array_equal(glisted, listed)


@pytest.mark.gpu
def test_gpu_fanout_closure_queue_trace(engine):
    """The ClosureQueueTest trace, one kernel launch per popClosureUntil call."""
    first, size = 0, 10
    trace = [(4, 0, 5), (4, 5, 0), (3, 4, 0), (10, -1, 0), (9, 5, 5), (1, 2, 0), (3, 4, 0)]
    for end, ret, popped in trace:
        st, fc, listed, cf, cs = engine.commit_fanout([end - 1], [end], [I64_MIN], [first], [size])
        assert (int(fc[0]), size - int(cs[0])) == (ret, popped)
        assert list(listed) == [0]
        first, size = int(cf[0]), int(cs[0])
    assert (first, size) == (10, 0)


@pytest.mark.gpu
def test_gpu_fanout_after_quorum_epoch_dev(engine):
    """Device chaining: quorum epoch output feeds the fan-out without a host round trip."""
    import torch

    from jraft_amd import workloads as W
    b = W.quorum_batch("C3", groups=20_000)
    G = b["pending_index"].shape[0]
    dev = torch.device("cuda", 0)
    t = {k: to_dev(np.ascontiguousarray(v.view(np.int64) if v.dtype == np.uint64 else v), dev)
         for k, v in b.items() if isinstance(v, np.ndarray)}
    committed = torch.empty(G, dtype=torch.int64, device=dev)
    status = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                            t["last_committed"], t["conf"], committed, status)
    rng = np.random.default_rng(7)
    la = b["last_committed"].copy()
    cq_first = b["pending_index"].copy()
    cq_size = (b["last_appended"] - b["pending_index"] + 1).astype(np.int64)
    la[rng.random(G) < 0.1] += 10_000
    d_la = to_dev(la, dev)
    d_cf = to_dev(cq_first, dev)
    d_cs = to_dev(cq_size, dev)
    fc = torch.empty(G, dtype=torch.int64, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    listed = torch.empty((G + 63) // 64, dtype=torch.int64, device=dev)
    num = torch.full((1,), 12345, dtype=torch.int32, device=dev)  # the launch resets it
    engine.commit_fanout_dev(t["last_committed"], committed, d_la, d_cf, d_cs, fc, st, listed, num)
    engine.synchronize()
    c = host_np(committed)
    seq_off = np.zeros(G + 1, np.uint64)
    adv = c > b["last_committed"]
    seq_off[1:] = np.cumsum(adv)
    est, efc, _, ecf, ecs, elisted = oracle_epoch(dict(seq_off=seq_off, seq=c[adv], last_applied=la,
                                                       cq_first=cq_first, cq_size=cq_size))
    assert np.array_equal(host_np(st), est)
    assert np.array_equal(host_np(fc), efc)
    assert np.array_equal(host_np(d_cf), ecf)
    assert np.array_equal(host_np(d_cs), ecs)
    from jraft_amd.engine import listed_ids
    assert int(num.item()) == len(elisted)
    assert np.array_equal(listed_ids(host_np(listed), G), elisted)
    assert (est == O.FAN_APPLY).sum() > G // 2


@pytest.mark.gpu
@pytest.mark.parametrize("G", [(1 << 20) + 37, (1 << 20) + 66])
def test_gpu_fanout_full_size_closed_form(engine, G):
    """C3-sized batch (1M groups): the kernel against the numpy closed form (the form the
    call-by-call replay pins above), with a non-multiple-of-64 tail: odd G (one group per lane)
    and even G (two per lane, fanout_pair; the last wave's second bitmap word partial)."""
    rng = np.random.default_rng(99)
    prev = rng.integers(0, 1 << 40, G).astype(np.int64)
    committed = prev + np.where(rng.random(G) < 0.8, rng.integers(1, 1024, G), 0)
    la = prev - rng.integers(0, 3, G)
    la[rng.random(G) < 0.03] += 1 << 20
    cf = prev + 1
    cs = np.where(rng.random(G) < 0.3, 0, 1024 + rng.integers(0, 8, G)).astype(np.int64)
    cs[rng.random(G) < 0.01] = 1  # some commits beyond the queue -> INVALID
    st, fc, listed, gcf, gcs = engine.commit_fanout(prev, committed, la, cf, cs)
    est, efc, ecf, ecs = closed_form(prev, committed, la, cf, cs)
    assert np.array_equal(st, est) and np.array_equal(fc, efc)
    assert np.array_equal(gcf, ecf) and np.array_equal(gcs, ecs)
    assert np.array_equal(listed, np.nonzero((est == O.FAN_APPLY) | (est == O.FAN_INVALID))[0])
    assert (est == O.FAN_INVALID).any() and (est == O.FAN_SKIP).any()
