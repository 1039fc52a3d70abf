"""GPU: the drop-in path end to end -- a C3-shaped multi-Raft series replayed through the C++
host mirror's BallotBox API (appendPendingTask / commitAt, sofa-jraft_amd/host) over the
resident device table, one GroupBatch::flush() per epoch (libjraft_drive.so).

Checked against (a) the oracle's Java-faithful BallotBox replays on a sample of groups and (b)
the stateless K-epoch kernel on every group, with a conf change inside the pending window of
some groups; and the upload is exactly the changed acks and queue sizes, the download exactly
the changed commits.
"""
import numpy as np
import pytest

from jraft_amd import workloads as W
from quorum_cases import series_replay
from devio import to_dev, host_np

pytestmark = pytest.mark.gpu


def _expected_counts(s, committed):
    """Records the mirror must ship per epoch (changed queue sizes of leaders + acks that moved
    a peer's match at or past pendingIndex) and groups whose commit moved."""
    K, P, G = s["match"].shape
    pi = s["pending_index"].copy()
    prev_c = s["last_committed"].copy()
    recs, changed = [], []
    for k in range(K):
        m = s["match"][k]
        if k == 0:
            recs.append(int((m >= pi).sum()))
        else:
            la_ch = s["last_appended"][k] != s["last_appended"][k - 1]
            moved = (m > s["match"][k - 1]) & (m >= pi)
            recs.append(int(la_ch.sum() + moved.sum()))
        c = committed[k]
        changed.append(int((c > prev_c).sum()))
        pi = np.where(c > prev_c, c + 1, pi)
        prev_c = c
    return recs, changed


@pytest.mark.parametrize("G,K,joint,active,threads,shards", [(20000, 5, 0.05, 0.5, 1, 1),
                                                             (4096, 4, 0.3, 1.0, 1, 1),
                                                             (50000, 4, 0.1, 0.8, 16, 1),
                                                             (50000, 4, 0.1, 0.8, 16, 2),
                                                             (4099, 4, 0.3, 1.0, 3, 3)])
def test_host_mirror_drives_series(engine, oracle, G, K, joint, active, threads, shards):
    """threads = 16: each epoch's calls come from 16 threads at once (group slices); the
    flush packs and delivers on its own worker threads (> 8192 changed groups).  shards > 1:
    the groups over that many engines in this process (ShardedGroupBatch, the last block
    ragged), committed read back from the published node-wide snapshot."""
    import torch
    from conftest import assert_unregistered, device_checkpoint

    from jraft_amd import drive
    s = W.host_series("C3", K, groups=G, joint_frac=joint, active=active)
    assert_unregistered(s, "before drive_epochs")
    committed, st = drive.drive_epochs(0, s, threads=threads, shards=shards)
    # (round 3 saw one "illegal memory access" in this test: the checkpoints name the step)
    device_checkpoint("after drive_epochs (the mirror's flushes, its engine destroyed)")
    assert_unregistered(s, "after drive_epochs")
    # (b) every group against the stateless K-epoch kernel with the same conf runs
    dev = torch.device("cuda:0")
    t = {}
    for k in ("match", "last_appended", "pending_index", "last_committed", "conf", "run_off",
              "run_start", "run_conf"):
        t[k] = to_dev(np.ascontiguousarray(s[k].view(np.int64) if s[k].dtype == np.uint64
                                                     else s[k]), dev)
        device_checkpoint(f"after the torch upload of {k} ({s[k].nbytes} B, pageable)")
    c = torch.empty((K, G), dtype=torch.int64, device=dev)
    sst = torch.empty((K, G), dtype=torch.uint8, device=dev)
    engine.quorum_epochs_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], c, sst, run_off=t["run_off"],
                             run_start=t["run_start"], run_conf=t["run_conf"])
    device_checkpoint("after quorum_epochs_dev")
    np.testing.assert_array_equal(committed, host_np(c))
    # (a) a sample of groups (all the joint ones among them) against the oracle
    rng = np.random.default_rng(1)
    joint_g = np.nonzero(s["switch_at"])[0]
    sub = np.unique(np.concatenate([rng.choice(G, 600, replace=False), joint_g[:200]]))
    ro = s["run_off"]
    sub_s = dict(match=s["match"][:, :, sub], last_appended=s["last_appended"][:, sub],
                 pending_index=s["pending_index"][sub], last_committed=s["last_committed"][sub],
                 conf=s["conf"][sub])
    cnt = (ro[sub + 1] - ro[sub]).astype(np.uint32)
    sub_s["run_off"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    idx = np.concatenate([np.arange(ro[g], ro[g + 1]) for g in sub])
    sub_s["run_start"] = s["run_start"][idx]
    sub_s["run_conf"] = s["run_conf"][idx]
    ce, _ = series_replay(oracle, sub_s, chunk=1024)
    np.testing.assert_array_equal(committed[:, sub], ce)
    assert (committed[-1] > committed[0]).sum() > G // 4
    # upload = changed acks + changed queue sizes (+ one header per group at the first
    # flush); download = the changed commits
    recs, changed = _expected_counts(s, committed)
    np.testing.assert_array_equal(st["records"], recs)
    # after the first flush (which sizes the threads' record buffers) the acks and queue sizes
    # go up as the order-free records written at call time, not as pack records
    assert (st["acks"][1:] == st["records"][1:]).all() and st["acks"][0] == 0
    np.testing.assert_array_equal(st["changed"], changed)
    assert st["states"][0] == G and (st["states"][1:] == 0).all()
    np.testing.assert_array_equal(st["h2d_bytes"], st["states"] * 96 + st["records"] * 8)
    # each shard's list total + the entries
    np.testing.assert_array_equal(st["d2h_bytes"], 4 * shards + st["changed"] * 8)


def test_flusher_latency_small():
    """The background flusher under steady load (GroupBatch::startFlusher): every entry is
    acked by all peers and then committed; onCommitted follows the quorum-completing ack
    within the policy's delay plus one epoch."""
    from jraft_amd import drive
    r = drive.drive_latency(0, groups=4096, peers=3, threads=4, seconds=1.0, max_delay_us=500,
                            max_dirty=1 << 14, flush_threads=2, pass_us=2000)
    assert r["entries"] > 4096 and r["commits"] > 0 and r["samples"] > 0
    assert r["flushes"] > 10
    assert r["p50_us"] < 50_000, r
