"""GPU: C1's commit half (BASELINE configs[0]: 1 Raft group x 3 peers, 1M appended entries).

The checksum half of C1 is checked at full size in test_gpu_crc.py; this file checks the
commit half the same way: one group whose pending window holds 1M
ballots, acked in 1024-entry chunks as the reference's BallotBoxTest-style replay does
(BallotBox.java:96-139 per chunk, Ballot.grant per entry), decided by

* the stateless epoch (jrq_quorum_epoch_dev, one launch for the whole 1M window),
* K epochs per launch with 1024 entries appended and acked per epoch (jrq_quorum_epochs_dev),
* the resident table (one header, one record per peer, one in-place epoch),

each bit-exact against the oracle's replay.
"""
import numpy as np
import pytest

from jraft_amd import Table, _lib, decode_changed
from jraft_amd import workloads as W
from quorum_cases import series_replay
from devio import to_dev, host_np

pytestmark = pytest.mark.gpu


def _dev(a, dev):
    return to_dev(a, dev)


def test_c1_commit_one_epoch(engine, oracle):
    b = W.quorum_batch("C1")
    assert b["match"].shape == (3, 1) and b["last_appended"][0] - b["pending_index"][0] + 1 == 1 << 20
    ce, se, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                           b["last_committed"], b["conf"], chunk=1024)
    c, s = engine.quorum_epoch(b["match"], b["pending_index"], b["last_appended"],
                               b["last_committed"], b["conf"])
    np.testing.assert_array_equal(c, ce)
    np.testing.assert_array_equal(s, se)
    assert ce[0] > b["last_committed"][0]  # the window commits


def test_c1_commit_k_epochs(engine, oracle):
    """8 epochs of C1 in one launch: 1024 entries appended per epoch, every follower's ack moving
    by up to 2048 entries, the group's state carried as BallotBox carries it."""
    import torch
    K = 8
    s = W.quorum_epoch_series("C1", K, step=1024)
    ce, se = series_replay(oracle, s, chunk=1024)
    dev = torch.device("cuda:0")
    d = {k: _dev(v, dev) for k, v in s.items()}
    c = torch.empty((K, 1), dtype=torch.int64, device=dev)
    st = torch.empty((K, 1), dtype=torch.uint8, device=dev)
    engine.quorum_epochs_dev(d["match"], d["pending_index"], d["last_appended"],
                             d["last_committed"], d["conf"], c, st)
    engine.synchronize()
    np.testing.assert_array_equal(host_np(c), ce)
    np.testing.assert_array_equal(host_np(st), se)
    assert (np.diff(ce[:, 0]) > 0).any()


def test_c1_commit_resident_table(engine, oracle):
    b = W.quorum_batch("C1")
    ce, _, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                          b["last_committed"], b["conf"], chunk=1024)
    pi, lc = b["pending_index"], b["last_committed"]
    st = Table.states(1)
    st["group"] = 0
    st["num_runs"] = 1
    st["flags"] = _lib.STATE_RESET_MATCH
    st["pending_index"] = pi
    st["last_appended"] = b["last_appended"]
    st["last_committed"] = lc
    st["run_conf"][:, 0] = b["conf"]
    recs = np.concatenate([_lib.rec([0], p, np.maximum(b["match"][p] - (pi - 1), 0))
                           for p in range(3)])
    t = Table(engine, 1, 3)
    try:
        t.update(st, recs)
        changed, _ = t.epoch()
        g, dlt = decode_changed(changed)
        assert list(g) == [0]
        assert pi[0] - 1 + dlt[0] == ce[0]
        t.check()
    finally:
        t.close()
