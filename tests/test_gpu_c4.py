"""GPU: BASELINE config C4 -- 8M Raft groups x 5 peers, joint consensus, sharded by groupId over
8 GPUs with an all-gather of the committed-index snapshot -- on the box's one GPU.

* test_c4_eight_shards_one_gpu: the eight 1M-group rank shards (group_offset = r * 1M, the
  seeds bench.py --gpus 8 uses) run one after another through the engine's quorum epoch inside
  jraft_amd.dist.ShardedEpochs (the loop bench.py runs), each publishing its shard with
  jrq_publish_committed_dev over a single-rank RCCL communicator into its rank-major slice of one
  node-wide snapshot; the snapshot is unpadded with the same layout code and checked against the
  oracle's BallotBox replay on 8 x 4096 sampled groups, plus lastCommitted <= committed <=
  lastAppended on all 8M groups.
* test_c4_ranks_as_processes: the same orchestration with one process per rank (world 2, both on
  cuda:0, gloo carrying the all-gather of host copies): each rank's engine decides its shard.

A communicator of several ranks needs one GPU per rank (RCCL refuses two ranks on one device);
the box has one, so jrq_rccl_init with nranks > 1 has not run here.
"""
import os
import socket

import numpy as np
import pytest
from devio import to_dev, host_np, host_t

pytestmark = pytest.mark.gpu

G_RANK = 1 << 20   # C4: 1M groups per GPU
WORLD = 8
SAMPLE = 4096


def _seed(cfg, e):
    from jraft_amd import workloads as W
    return (W.SEED_BASE ^ int(cfg[1])) + 7919 * e   # bench.py leg_quorum's epoch buffers


def _check_shard(oracle, b, got, st, rank):
    """Sampled groups vs the replay; the range property on every group of the shard."""
    idx = np.random.default_rng(rank).choice(len(got), SAMPLE, replace=False)
    ce, se, _ = oracle.quorum_epoch_replay(b["match"][:, idx], b["pending_index"][idx],
                                           b["last_appended"][idx], b["last_committed"][idx],
                                           b["conf"][idx], chunk=1024)
    np.testing.assert_array_equal(got[idx], ce, err_msg=f"rank {rank}")
    np.testing.assert_array_equal(st[idx], se, err_msg=f"rank {rank}")
    lc, la = b["last_committed"], b["last_appended"]
    assert ((got >= lc) & (got <= np.maximum(la, lc))).all(), f"rank {rank}: commit out of range"
    return int((got > lc).sum())


def test_c4_eight_shards_one_gpu(oracle):
    import torch

    from jraft_amd import Engine
    from jraft_amd import dist as D
    from jraft_amd import workloads as W
    dev = torch.device("cuda:0")
    Gtot = G_RANK * WORLD
    k = D.per_rank(Gtot, WORLD)
    assert k == G_RANK
    snapshot = torch.full((k * WORLD,), -7, dtype=torch.int64, device=dev)
    K = 2   # epochs per rank, each on its own epoch buffer (bench.py cycles 6)
    with Engine(0, max_groups=G_RANK, max_peers=5) as eng:
        eng.rccl_init(1, 0, Engine.rccl_unique_id())
        assert eng.rccl_nranks() == 1
        committed_total = 0
        for rank in range(WORLD):
            batches = [W.quorum_batch("C4", groups=G_RANK, group_offset=rank * G_RANK,
                                      seed=_seed("C4", e)) for e in range(K)]
            dbs = [{n: to_dev(v, dev) for n, v in b.items()} for b in batches]
            local = torch.full((k,), -1, dtype=torch.int64, device=dev)
            status = torch.empty(G_RANK, dtype=torch.uint8, device=dev)

            def epoch_fn(i, out):
                t = dbs[i % K]
                eng.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                                     t["last_committed"], t["conf"], out, status)

            def allgather(send, recv, rank=rank):
                # a single-rank communicator gathers the rank's own block: its slice of the
                # rank-major node snapshot (an 8-rank all-gather writes the other 7 as well)
                eng.publish_committed_dev(send, recv[rank * k:(rank + 1) * k])

            se = D.ShardedEpochs(Gtot, WORLD, rank, epoch_fn, allgather, local, snapshot)
            assert (se.lo, se.hi) == (rank * G_RANK, (rank + 1) * G_RANK)
            for _ in range(K):
                se.step()
            eng.synchronize()
            assert se.published == K
            got = host_np(local)
            committed_total += _check_shard(oracle, batches[(K - 1) % K], got,
                                            host_np(status), rank)
        snap = D.unpad_snapshot(host_np(snapshot), Gtot, WORLD)
    assert snap.shape == (Gtot,)
    # every rank's block landed in groupId order: re-derive it from the shards' own seeds
    for rank in range(WORLD):
        b = W.quorum_batch("C4", groups=G_RANK, group_offset=rank * G_RANK, seed=_seed("C4", K - 1))
        blk = snap[rank * G_RANK:(rank + 1) * G_RANK]
        lc, la = b["last_committed"], b["last_appended"]
        assert ((blk >= lc) & (blk <= np.maximum(la, lc))).all()
        idx = np.random.default_rng(100 + rank).choice(G_RANK, SAMPLE, replace=False)
        ce, _, _ = oracle.quorum_epoch_replay(b["match"][:, idx], b["pending_index"][idx],
                                              b["last_appended"][idx], lc[idx], b["conf"][idx],
                                              chunk=1024)
        np.testing.assert_array_equal(blk[idx], ce, err_msg=f"snapshot block of rank {rank}")
    assert committed_total > WORLD * G_RANK // 2  # the C4 inputs commit most groups


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_proc(rank, world, port, G, K, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "sofa-jraft_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from jraft_amd import Engine
    from jraft_amd import dist as D
    from jraft_amd import workloads as W
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        Gtot = G * world
        k = D.per_rank(Gtot, world)
        with Engine(0, max_groups=G, max_peers=5) as eng:
            dbs = [{n: to_dev(v, dev) for n, v in
                    W.quorum_batch("C4", groups=G, group_offset=rank * G,
                                   seed=_seed("C4", e)).items()} for e in range(K)]
            local = torch.full((k,), -1, dtype=torch.int64, device=dev)
            status = torch.empty(G, dtype=torch.uint8, device=dev)
            snapshot = torch.empty(k * world, dtype=torch.int64)

            def epoch_fn(i, out):
                t = dbs[i % K]
                eng.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                                     t["last_committed"], t["conf"], out, status)

            def allgather(send, recv):
                eng.synchronize()
                dist.all_gather_into_tensor(recv, host_t(send))

            se = D.ShardedEpochs(Gtot, world, rank, epoch_fn, allgather, local, snapshot)
            for _ in range(K):
                se.step()
            if rank == 0:
                q.put(se.snapshot_groups(lambda t: t.numpy()).copy())
    finally:
        dist.destroy_process_group()


def test_c4_ranks_as_processes(oracle):
    """One process per rank, both ranks' engines on cuda:0, gloo for the all-gather: the
    snapshot equals the per-shard oracle replays in groupId order."""
    import torch.multiprocessing as mp

    from jraft_amd import workloads as W
    world, G, K = 2, 1 << 18, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_proc, args=(r, world, port, G, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    snap = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        b = W.quorum_batch("C4", groups=G, group_offset=rank * G, seed=_seed("C4", K - 1))
        idx = np.random.default_rng(rank).choice(G, SAMPLE, replace=False)
        ce, _, _ = oracle.quorum_epoch_replay(b["match"][:, idx], b["pending_index"][idx],
                                              b["last_appended"][idx], b["last_committed"][idx],
                                              b["conf"][idx], chunk=1024)
        np.testing.assert_array_equal(snap[rank * G:(rank + 1) * G][idx], ce)
