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
