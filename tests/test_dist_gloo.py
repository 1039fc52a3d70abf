"""CPU, world_size 2 (gloo): groupId sharding + committed-snapshot all-gather.

Each rank evaluates only its contiguous block of groups (the oracle stands in for
the GPU kernel here: this test is about the host-side sharding/publication logic,
which bench.py and the RCCL path share), pads, all-gathers, un-pads; the
snapshot must equal the unsharded evaluation in groupId order.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from jraft_amd import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, G, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "sofa-jraft_amd"), os.path.join(root, "oracle"),
              os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import jraft_oracle as O
    from jraft_amd import dist as D
    from quorum_cases import random_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = random_batch(1234, G, 5)
        mine = D.shard_batch(full, G, world, rank)
        c, s, _ = O.quorum_epoch_replay(mine["match"], mine["pending_index"], mine["last_appended"],
                                        mine["last_committed"], mine["conf"], mine["run_off"],
                                        mine["run_start"], mine["run_conf"], chunk=5)
        send = torch.from_numpy(D.pad_local(c, G, world))
        recv = torch.empty(send.numel() * world, dtype=torch.int64)
        dist.all_gather_into_tensor(recv, send)
        snap = D.unpad_snapshot(recv.numpy(), G, world)
        if rank == 0:
            q.put(snap)
    finally:
        dist.destroy_process_group()


def _engine_worker(rank, world, port, G, K, every, q):
    """The bench's orchestration (jraft_amd.dist.ShardedEpochs) with the oracle standing in for
    the epoch kernel and gloo for RCCL: K epochs of a C3-shaped series, publish every `every`."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "sofa-jraft_amd"), os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import jraft_oracle as O
    from jraft_amd import dist as D
    from jraft_amd import workloads as W
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = D.shard_bounds(G, world, rank)
        series = W.quorum_epoch_series("C3", K, groups=G)
        state = {"pi": series["pending_index"][lo:hi].copy(), "lc": series["last_committed"][lo:hi].copy()}

        def epoch_fn(i, local):
            c, _, _ = O.quorum_epoch_replay(series["match"][i][:, lo:hi], state["pi"],
                                            series["last_appended"][i][lo:hi], state["lc"],
                                            series["conf"][lo:hi], chunk=1024)
            state["pi"] = np.where((state["pi"] != 0) & (c > state["lc"]), c + 1, state["pi"])
            state["lc"] = c
            local[: hi - lo] = torch.from_numpy(c)

        k = D.per_rank(G, world)
        local = torch.full((k,), -1, dtype=torch.int64)
        snap = torch.empty(k * world, dtype=torch.int64)
        se = D.ShardedEpochs(G, world, rank, epoch_fn,
                             lambda send, recv: dist.all_gather_into_tensor(recv, send), local,
                             snap, publish_every=every)
        snaps = []
        for _ in range(K):
            before = se.published
            se.step()
            if se.published != before:
                snaps.append(se.snapshot_groups(lambda t: t.numpy()).copy())
        if rank == 0:
            q.put((se.published, snaps))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("G,K,every", [(1001, 4, 1), (513, 5, 2)])
def test_sharded_epochs_orchestration(oracle, G, K, every):
    """bench.py --gpus N's loop (ShardedEpochs) at world 2: every published snapshot equals the
    unsharded oracle series at that epoch; publications happen every `every` epochs."""
    from quorum_cases import series_replay
    from jraft_amd import workloads as W
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, world, port, G, K, every, q))
             for r in range(world)]
    for p in procs:
        p.start()
    published, snaps = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert published == K // every == len(snaps)
    series = W.quorum_epoch_series("C3", K, groups=G)
    expect, _ = series_replay(oracle, series, chunk=1024)
    for j, snap in enumerate(snaps):
        np.testing.assert_array_equal(snap, expect[(j + 1) * every - 1])


@pytest.mark.parametrize("G", [1001, 64])
def test_sharded_snapshot_equals_unsharded(oracle, G):
    from quorum_cases import random_batch
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, q)) for r in range(world)]
    for p in procs:
        p.start()
    snap = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = random_batch(1234, G, 5)
    c, _, _ = oracle.quorum_epoch_replay(full["match"], full["pending_index"],
                                         full["last_appended"], full["last_committed"],
                                         full["conf"], full["run_off"], full["run_start"],
                                         full["run_conf"], chunk=5)
    np.testing.assert_array_equal(snap, c)


def test_shard_bounds_cover_all_groups():
    for G in (0, 1, 7, 8, 1 << 20, 8 << 20):
        for world in (1, 2, 4, 8):
            seen = 0
            for r in range(world):
                lo, hi = D.shard_bounds(G, world, r)
                assert lo == min(G, seen) and hi >= lo
                seen = hi
            assert seen == G


def test_pad_unpad_roundtrip():
    G, world = 10, 4
    full = np.arange(G, dtype=np.int64) * 3
    gathered = np.concatenate([D.pad_local(full[slice(*D.shard_bounds(G, world, r))], G, world)
                               for r in range(world)])
    np.testing.assert_array_equal(D.unpad_snapshot(gathered, G, world), full)


def _publish_choice_worker(rank, world, port, fail_ranks, q):
    """jraft_amd.dist.choose_publish as bench.py's leg_quorum calls it, with the RCCL init
    replaced by a stand-in that fails on `fail_ranks` (the injected failure) and gloo as the
    process group."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "sofa-jraft_amd"))
    import torch
    import torch.distributed as dist

    from jraft_amd import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def rccl_init():
            if rank in fail_ranks:
                raise RuntimeError("JRQ_E_RCCL: injected ncclCommInitRank failure")
            return world

        used = []

        def rccl_publish(send, recv):
            used.append("rccl")
            dist.all_gather_into_tensor(recv, send)

        def pg_publish(send, recv):
            used.append("pg")
            dist.all_gather_into_tensor(recv, send)

        def agree(ok):
            t = torch.tensor([1 if ok else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            return bool(t.item())

        fn, info = D.choose_publish(world, "nccl", rccl_init, rccl_publish, pg_publish, agree)
        G = 37
        k = D.per_rank(G, world)
        lo, hi = D.shard_bounds(G, world, rank)
        local = torch.from_numpy(D.pad_local(np.arange(lo, hi, dtype=np.int64) * 5, G, world))
        snap = torch.empty(k * world, dtype=torch.int64)
        se = D.ShardedEpochs(G, world, rank, lambda i, out: None, fn, local, snap)
        se.step()
        q.put((rank, info, used, se.snapshot_groups(lambda t: t.numpy()).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_ranks,expect_rccl", [((), True), ((1,), False), ((0, 1), False)])
def test_publish_falls_back_when_rccl_init_fails(fail_ranks, expect_rccl):
    """VERDICT r05 missing #3 / weak #6: a failed RCCL communicator init on any rank makes every
    rank publish through the process group (the run still prints its line), the error is
    recorded, and rccl_nranks is None whenever no communicator exists."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_publish_choice_worker, args=(r, world, port, fail_ranks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (i, u, s)) for r, i, u, s in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        info, used, snap = res[r]
        assert snap == [g * 5 for g in range(37)]
        assert info["ranks"] == world
        if expect_rccl:
            assert used == ["rccl"] and info["rccl_nranks"] == world and info["rccl_error"] is None
            assert "RCCL" in info["publish_via"]
        else:
            assert used == ["pg"] and info["rccl_nranks"] is None
            assert "init failed" in info["publish_via"] and info["rccl_error"]
            if r in fail_ranks:
                assert "injected" in info["rccl_error"]


def test_publish_choice_single_rank_and_gloo():
    fn, info = D.choose_publish(1, "nccl", None, None, None, None)
    assert fn is None and info["rccl_nranks"] is None and info["ranks"] == 1
    pg = object()
    fn, info = D.choose_publish(2, "gloo", None, None, pg, None)
    assert fn is pg and info["rccl_nranks"] is None and "gloo" in info["publish_via"]
