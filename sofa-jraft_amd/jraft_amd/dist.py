"""Group sharding across the GPUs of one node and the committed-index snapshot layout.

Raft groups are independent (one BallotBox per NodeImpl, jraft-core/.../core/
NodeImpl.java:829-836; multi-Raft = many NodeImpls, rheakv StoreEngine.java:93),
so groups shard by contiguous, dense groupId blocks with no data-path exchange.
The only collective is the all-gather that publishes every rank's committed[]
as one node-wide snapshot: libjrq's jrq_publish_committed_dev
(RCCL over xGMI) on GPUs; any torch.distributed backend (gloo in CPU tests)
can run the same layout.

All-gather needs equal counts per rank, so every rank contributes
`per_rank = ceil(G / world)` slots (the last block is padded) and the snapshot
is rank-major: slot r * per_rank + i holds group lo_r + i.
"""
from __future__ import annotations

import numpy as np


def per_rank(G: int, world: int) -> int:
    return -(-G // world) if G else 0


def shard_bounds(G: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of the contiguous groupId block owned by `rank`."""
    if not 0 <= rank < world:
        raise ValueError("rank outside world")
    k = per_rank(G, world)
    lo = min(G, rank * k)
    return lo, min(G, lo + k)


def pad_local(committed_local: np.ndarray, G: int, world: int, fill: int = -1) -> np.ndarray:
    """The rank's all-gather send buffer: its committed[] padded to per_rank slots."""
    k = per_rank(G, world)
    out = np.full(k, fill, dtype=np.int64)
    out[: len(committed_local)] = committed_local
    return out


def unpad_snapshot(gathered: np.ndarray, G: int, world: int) -> np.ndarray:
    """Rank-major gathered buffer (world * per_rank) -> committed[G] in groupId order."""
    k = per_rank(G, world)
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(G, world, r)
        parts.append(gathered[r * k: r * k + (hi - lo)])
    return np.concatenate(parts) if parts else np.zeros(0, np.int64)


def shard_batch(batch: dict, G: int, world: int, rank: int) -> dict:
    """Slice a group batch (match [P][G] + per-group arrays) to the rank's block."""
    lo, hi = shard_bounds(G, world, rank)
    out = {}
    for k, v in batch.items():
        if v is None:
            out[k] = None
        elif k == "match":
            out[k] = np.ascontiguousarray(v[:, lo:hi])
        elif k in ("run_off", "run_start", "run_conf"):
            continue  # run tables are re-based by shard_runs
        else:
            out[k] = np.ascontiguousarray(v[lo:hi])
    if batch.get("run_off") is not None:
        ro = batch["run_off"]
        a, b = int(ro[lo]), int(ro[hi])
        out["run_off"] = (ro[lo:hi + 1] - a).astype(np.uint32)
        out["run_start"] = np.ascontiguousarray(batch["run_start"][a:b])
        out["run_conf"] = np.ascontiguousarray(batch["run_conf"][a:b])
    return out
