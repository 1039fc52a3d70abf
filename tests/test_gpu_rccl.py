"""GPU: the committed-snapshot publication through libjrq's own RCCL communicator.

The box has one GPU, so this runs a single-rank communicator (all-gather of one shard);
the multi-rank layout is covered by tests/test_dist_gloo.py and bench.py --gpus N."""
import numpy as np
import pytest
from devio import host_np

pytestmark = pytest.mark.gpu


def test_single_rank_publish(engine):
    import torch
    from jraft_amd import Engine
    uid = Engine.rccl_unique_id()
    assert len(uid) == 128
    engine.rccl_init(1, 0, uid)
    dev = torch.device("cuda:0")
    local = torch.arange(1000, dtype=torch.int64, device=dev) * 7 - 3
    glob = torch.full((1000,), -1, dtype=torch.int64, device=dev)
    engine.publish_committed_dev(local, glob)
    engine.synchronize()
    np.testing.assert_array_equal(host_np(glob), host_np(local))


def test_publish_without_init_is_state_error():
    import torch
    from jraft_amd import Engine, JrqError
    dev = torch.device("cuda:0")
    with Engine(0) as e:
        x = torch.zeros(4, dtype=torch.int64, device=dev)
        with pytest.raises(JrqError) as ei:
            e.publish_committed_dev(x, x)
        assert ei.value.code == -6
