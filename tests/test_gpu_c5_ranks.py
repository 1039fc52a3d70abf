"""GPU: BASELINE config C5 at N > 1 -- 64k RheaKV-style regions x 3 replicas x 16 KiB entries per
GPU, regions sharded by regionId (StoreEngine.java:93 / RegionEngine.java:126-127 shard regions as
groups shard) -- as two rank shards run one after another on the box's one GPU through bench.py's
own C5 leg (`leg_c5`, the code `bench.py --gpus N` runs on every rank).  Each shard has its own
payload seed and region offset (rank * 64k) and is checked against the oracle: every entry's
LogEntry checksum and corrupt flag (1/1024 flipped), and the commit of every one of its 64k
groups against the BallotBox replay.
"""
import os
import sys
import types

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c5_two_rank_shards_one_gpu(engine):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from jraft_amd import workloads as W

    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    args = types.SimpleNamespace(steps=3, warmup=1, no_cpu=False)
    payload_digests, commits = [], []
    old = bench.WARM_MS
    bench.WARM_MS = 5.0  # the timing is not what this test checks
    try:
        with torch.cuda.stream(stream):
            engine.use_stream(stream.cuda_stream)
            for rank in range(2):
                ctx = bench.Ctx(engine, stream, dev, 2, rank, args)
                ctx.gather = lambda x: [x]  # one process stands in for each rank in turn
                crc, step, state = bench.leg_c5(ctx, args, lambda: None, lambda x: x)
                assert crc["bit_exact_vs_oracle"] is True, f"rank {rank}: CRC verify"
                assert crc["offsets_path"]["bit_exact_vs_oracle"] is True, f"rank {rank}: offsets"
                assert step["bit_exact_vs_oracle"] is True, f"rank {rank}: verify + commit"
                assert crc["per_rank_bit_exact"] == [True]
                d, eb, expected, flip, out = state
                payload_digests.append(int(np.bitwise_xor.reduce(expected)))
                commits.append(W.quorum_batch("C5", group_offset=rank * W.CONFIGS["C5"]["groups"]))
                del d, state
                torch.cuda.synchronize()
    finally:
        bench.WARM_MS = old
        engine.use_stream(None)
    # the two shards are different data (their own payloads and groups), not one shard twice
    assert payload_digests[0] != payload_digests[1]
    assert not np.array_equal(commits[0]["match"], commits[1]["match"])
