"""The leader tick (jrq_leader_tick[_dev]): the lease check (NodeImpl.checkDeadNodes0 /
handleStepDownTimeout, NodeImpl.java:1970-2016) and the ReadIndex heartbeat round
(ReadIndexHeartbeatResponseClosure, :1246-1291) of the same leader groups in one launch.
Checked against the two oracle restatements (jo_lease_check, jo_readindex_round) on the same
inputs: the pair kernel (aligned, even and odd G), the one-group fallback (unaligned device
pointers), the lease check alone (no ReadIndex arrays) and the argument checks."""
import numpy as np
import pytest

from test_lease import random_lease_batch
from test_readindex import random_rounds
from devio import to_dev, host_np

pytestmark = pytest.mark.gpu


def _batch(seed, G, P):
    ts, conf, self_slot, now, to, lead = random_lease_batch(seed, G, P)
    # the ReadIndex rounds over the lease batch's own confs and self slots (random_rounds is a
    # Python loop: at most 4096 distinct rounds, tiled)
    _, _, order, okm, _ = random_rounds(seed + 1000, min(G, 4096), P)
    rep = -(-G // len(order))
    return ts, conf, self_slot, now, to, lead, np.tile(order, rep)[:G], np.tile(okm, rep)[:G]


def _expect(oracle, ts, conf, self_slot, now, to, lead, order, okm, P):
    ok, l2, dead = oracle.lease_check(ts, conf, self_slot, now, to, lead)
    ri = oracle.readindex_quorum(conf, self_slot, order, okm, P)
    return ok, l2, dead, ri


@pytest.mark.parametrize("P,G", [(1, 4001), (3, 20000), (5, 20001), (8, 3), (9, 4097), (16, 20000)])
def test_tick_matches_both_oracles(engine, oracle, P, G):
    ts, conf, self_slot, now, to, lead, order, okm = _batch(P, G, P)
    e = _expect(oracle, ts, conf, self_slot, now, to, lead, order, okm, P)
    g = engine.leader_tick(ts, conf, self_slot, now, to, lead, order, okm)
    for name, a, b in zip(("ok", "lease_start", "dead", "readindex"), g, e):
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert {0, 1, 2} <= set(np.unique(e[3])) or G < 100 or P < 3  # (P <= 2: quorum <= 1 answers at once)


@pytest.mark.parametrize("P", [3, 5])
def test_tick_lease_alone(engine, oracle, P):
    ts, conf, self_slot, now, to, lead, _, _ = _batch(40 + P, 9999, P)
    ok, l2, dead, ri = engine.leader_tick(ts, conf, self_slot, now, to, lead)
    assert ri is None
    e = oracle.lease_check(ts, conf, self_slot, now, to, lead)
    for a, b in zip((ok, l2, dead), e):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("off", [0, 1])
def test_tick_dev_aligned_and_unaligned(engine, oracle, off):
    """Device pointers on the 16-B grid (the pair kernel) and one element off it (the one-group
    kernels, the lease then the ReadIndex launch), 1M groups x 5 peers."""
    import torch
    P, G = 5, (1 << 20) + 1
    ts, conf, self_slot, now, to, lead, order, okm = _batch(77, G, P)
    dev = torch.device("cuda:0")
    T = lambda a: to_dev(np.ascontiguousarray(a), dev)  # noqa: E731
    # ts with a row stride of G + 1 (even when G is odd: the pair kernel's condition)
    ld = G + 1
    tsd = torch.zeros((P, ld), dtype=torch.int64, device=dev)
    tsd[:, off:off + G - off] = T(ts[:, off:])
    c = T(conf.view(np.int64))
    s = T(self_slot)
    o = T(order.view(np.int64))
    k = T(okm.view(np.int16))
    L = T(lead)
    ok = torch.zeros(G, dtype=torch.uint8, device=dev)
    dead = torch.zeros(G, dtype=torch.int16, device=dev)
    ri = torch.zeros(G, dtype=torch.uint8, device=dev)
    engine.leader_tick_dev(tsd[:, off:], c[off:], s[off:], now, to, ok[off:], L[off:], dead[off:],
                           o[off:], k[off:], ri[off:])
    torch.cuda.synchronize()
    sl = slice(off, None)
    e = _expect(oracle, ts[:, sl], conf[sl], self_slot[sl], now, to, lead[sl], order[sl], okm[sl], P)
    np.testing.assert_array_equal(host_np(ok)[sl], e[0])
    np.testing.assert_array_equal(host_np(L)[sl], e[1])
    np.testing.assert_array_equal(host_np(dead).view(np.uint16)[sl], e[2])
    np.testing.assert_array_equal(host_np(ri)[sl], e[3])


def test_tick_argument_checks(engine):
    import ctypes

    from jraft_amd import _lib
    L = _lib.load()
    ts = np.zeros((3, 4), np.int64)
    conf = np.zeros(4, np.uint64)
    s = np.zeros(4, np.uint8)
    ok = np.zeros(4, np.uint8)
    lead = np.zeros(4, np.int64)
    order = np.zeros(4, np.uint64)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    # order without ok_mask / result: refused
    rc = L.jrq_leader_tick(engine._h, p(ts), 4, 3, p(conf), p(s), 4, 0, 1, p(ok), p(lead), None,
                           p(order), None, None)
    assert rc == -1
    # ld < G, num_peers 0 / 17: refused
    assert L.jrq_leader_tick(engine._h, p(ts), 3, 3, p(conf), p(s), 4, 0, 1, p(ok), p(lead), None,
                             None, None, None) == -1
    assert L.jrq_leader_tick(engine._h, p(ts), 4, 0, p(conf), p(s), 4, 0, 1, p(ok), p(lead), None,
                             None, None, None) == -1
    assert L.jrq_leader_tick(engine._h, p(ts), 4, 17, p(conf), p(s), 4, 0, 1, p(ok), p(lead), None,
                             None, None, None) == -1
