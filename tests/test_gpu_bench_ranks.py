"""GPU: bench.py's N > 1 orchestration run as a whole, before the driver's 8-GPU scaling run does.

The driver launches `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
(one rank per GPU over RCCL).  This box has one GPU, and RCCL refuses two ranks on one device,
so the test runs the same main() as two ranks on cuda:0 with the process group on gloo
(`--dist-backend gloo --one-device`): process-group setup, the rank-sharded C4 epochs through
ShardedEpochs with the snapshot all-gathered every epoch (through host copies instead of
jrq_publish_committed_dev), barriers and max-over-ranks timing, the per-rank C5 shards, the
gathers of per-rank rates and parity verdicts, and rank 0's line.  The only piece of the
8-GPU run it does not execute is jrq_rccl_init with nranks > 1.
Groups shard by groupId as regions shard in RheaKV (StoreEngine.java:93).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_gpu(tmp_path):
    detail = tmp_path / "detail.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "1",
           "--legs", "quorum,C5", "--groups-per-gpu", str(1 << 18), "--dist-backend", "gloo",
           "--one-device", "--detail", str(detail)]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints exactly one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "C4" in line["config"]["workload"]
    mg = line["multi_gpu"]
    # no RCCL communicator exists under gloo: the line says so
    assert mg["rccl_nranks"] is None and mg["ranks"] == 2 and "gloo" in mg["publish_via"]
    assert mg["kernel_only_ms"] > 0 and mg["publish_ms"] is not None
    assert line["bit_exact_vs_oracle_4096_groups"] is True
    crc = line["crc64"]
    assert len(crc["per_rank_GBps"]) == 2 and all(v > 0 for v in crc["per_rank_GBps"])
    assert crc["per_rank_bit_exact"] == [True, True]
    full = json.loads(detail.read_text())
    assert full["C5"]["per_rank_bit_exact"] == [True, True]
    assert full["crc64"]["bit_exact_vs_oracle"] is True
    # the published snapshot covers both shards: 2 x 2^18 groups
    assert full["multi_gpu"]["snapshot_bytes"] == 8 * 2 * (1 << 18)
