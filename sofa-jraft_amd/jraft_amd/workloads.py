"""Seeded synthetic workloads for BASELINE.json's configs.

splitmix64 counter streams with seed 0x6A52414654 ^ config_id, vectorised in
numpy, so tests, bench.py and the CPU baseline see identical inputs.

  C1  1 group x 3 peers, 1M DATA entries x 256 B, pendingIndex 1, acks in 1024-entry chunks
  C2  10k groups x 3 peers x 1k pending, stable conf
  C3  1M groups x 5 peers, joint consensus (old 3 of the 5 + new 5)
  C4  C3 with 8M groups sharded by contiguous groupId blocks (1M per GPU)
  C5  64k regions x 3 replicas, one 16 KiB DATA entry per region per epoch,
      CRC64 verify (1/1024 corrupted) + quorum commit
"""
from __future__ import annotations

import numpy as np

from ._lib import conf_word

SEED_BASE = 0x6A52414654
GAMMA = np.uint64(0x9E3779B97F4A7C15)
ENTRY_TYPE_DATA = 2  # EnumOutter.EntryType.ENTRY_TYPE_DATA (jraft-core/.../entity/EnumOutter.java:46-48)

CONFIGS = {
    "C1": dict(groups=1, peers=3, pending=1 << 20, entry_bytes=256),
    "C2": dict(groups=10_000, peers=3, pending=1024),
    "C3": dict(groups=1 << 20, peers=5, pending=1024, joint=True),
    "C4": dict(groups=8 << 20, peers=5, pending=1024, joint=True),
    "C5": dict(groups=64 << 10, peers=3, pending=1, entry_bytes=16 << 10),
}


def splitmix64(seed: int, n: int, stream: int = 0) -> np.ndarray:
    """n outputs of splitmix64 seeded with `seed`, sub-stream `stream` (counter based)."""
    with np.errstate(over="ignore"):
        s = np.uint64((seed + stream * 0xD1B54A32D192ED03) & (2**64 - 1))
        z = s + (np.arange(1, n + 1, dtype=np.uint64) * GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed, n, lo, hi, stream):
    """Integers in [lo, hi) (hi - lo < 2^40)."""
    r = splitmix64(seed, n, stream)
    return (lo + (r % np.uint64(hi - lo)).astype(np.int64)).astype(np.int64)


def random_bytes(seed, nbytes, stream=99) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8, stream)
    return words.view(np.uint8)[:nbytes].copy()


def quorum_batch(cfg: str, groups: int | None = None, seed: int | None = None,
                 group_offset: int = 0):
    """Quorum inputs of one epoch for C2/C3/C4/C5-shaped group batches.

    Returns dict(match[P][G], pending_index, last_appended, last_committed, conf).
    `group_offset` selects a contiguous groupId shard (C4 sharding) with identical
    values to the unsharded batch."""
    c = CONFIGS[cfg]
    G = c["groups"] if groups is None else groups
    P = c["peers"]
    pend = c.get("pending", 1024)
    seed = (SEED_BASE ^ int(cfg[1])) if seed is None else seed
    # per-group values depend only on the global group id
    gid = np.arange(group_offset, group_offset + G, dtype=np.uint64)

    def stream_at(stream, lo, hi):
        # counter-based: value k of a stream = splitmix64 at counter gid (vectorised)
        with np.errstate(over="ignore"):
            s = np.uint64((seed + stream * 0xD1B54A32D192ED03) & (2**64 - 1))
            z = s + (gid + np.uint64(1)) * GAMMA
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
        return (lo + (z % np.uint64(hi - lo)).astype(np.int64)).astype(np.int64)

    pi = stream_at(1, 1, 1 << 40)
    la = pi + (pend - 1)
    lc = pi - 1
    match = np.empty((P, G), dtype=np.int64)
    match[0] = la  # leader's own disk-stable ack (LeaderStableClosure, NodeImpl.java:1147-1163)
    for p in range(1, P):
        match[p] = pi - 1 + stream_at(10 + p, 0, pend + 1)
    if c.get("joint"):
        # ~1/8 of groups have one lagging follower with no ack in this epoch
        lag = stream_at(30, 0, 8) == 0
        who = stream_at(31, 1, P)
        rows = np.where(lag)[0]
        match[who[rows], rows] = pi[rows] - 1 - stream_at(32, 0, 1000)[rows]
        new_mask = (1 << P) - 1
        # old conf = 3 of the 5 slots (C(5,3) = 10 choices), JRQ_CONF with quorums 3 / 2
        combos = [m for m in range(32) if bin(m).count("1") == 3]
        old = np.array(combos, dtype=np.uint64)[stream_at(33, 0, len(combos))]
        conf = (np.uint64(conf_word(new_mask)) & np.uint64(0xFFFF)) | (old << np.uint64(16)) | \
            (np.uint64(3) << np.uint64(32)) | (np.uint64(2) << np.uint64(40))
    else:
        conf = np.full(G, conf_word((1 << P) - 1), dtype=np.uint64)
    return dict(match=match, pending_index=pi, last_appended=la, last_committed=lc,
                conf=conf.astype(np.uint64))


def to_tiles(match, pending_index, last_appended, last_committed, conf) -> np.ndarray:
    """A quorum batch in the resident table's tile layout (include/jrq.h jrq_group_tiles):
    tiles of 256 groups, each holding match[0..P-1], pending_index, last_appended,
    last_committed, conf as 256-word rows; int64 words, G rounded up to whole tiles (pad
    groups: all zero, not leaders)."""
    match = np.asarray(match)
    P, G = match.shape[0], match.shape[1]
    nt = (G + 255) // 256
    rows = np.zeros((P + 4, nt * 256), np.int64)
    rows[:P, :G] = match[:, :G]
    rows[P, :G] = pending_index
    rows[P + 1, :G] = last_appended
    rows[P + 2, :G] = last_committed
    rows[P + 3, :G] = np.asarray(conf).view(np.int64)
    return np.ascontiguousarray(rows.reshape(P + 4, nt, 256).transpose(1, 0, 2)).reshape(-1)


def entry_batch(n_entries: int, entry_bytes: int, seed: int, first_index: int = 1,
                term: int = 1, corrupt_every: int = 0):
    """n DATA LogEntries of `entry_bytes` random bytes each (C1/C5 payload shape)."""
    payload = random_bytes(seed, n_entries * entry_bytes)
    offsets = np.arange(n_entries + 1, dtype=np.uint64) * np.uint64(entry_bytes)
    etype = np.full(n_entries, ENTRY_TYPE_DATA, dtype=np.uint8)
    index = np.arange(first_index, first_index + n_entries, dtype=np.int64)
    terms = np.full(n_entries, term, dtype=np.int64)
    return dict(payload=payload, offsets=offsets, etype=etype, index=index, term=terms,
                corrupt_every=corrupt_every)


def ragged_offsets(seed: int, n: int, max_len: int, start: int = 0, zero_frac: float = 0.05):
    """Monotone offsets with random lengths in [0, max_len], some zero-length entries."""
    lens = uniform(seed, n, 0, max_len + 1, stream=7)
    z = (splitmix64(seed, n, 8) % np.uint64(1000)).astype(np.float64) / 1000.0 < zero_frac
    lens[z] = 0
    off = np.zeros(n + 1, dtype=np.uint64)
    off[0] = start
    off[1:] = start + np.cumsum(lens).astype(np.uint64)
    return off


# ------------------------------------------------ stored V2 records (read path) --

V2_HEADER = bytes([0xBB, 0xD2, 0x01, 0, 0, 0])  # LogEntryV2CodecFactory.java:52-60


def pb_varint(v: int) -> bytes:
    """protobuf varint of a 64-bit two's complement integer."""
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if not v:
            out.append(b)
            return bytes(out)
        out.append(b | 0x80)


def v2_records(etype, index, term, payload, offsets, checksum):
    """DATA entries as V2Encoder writes them (V2Encoder.java:76-130, field order of the
    generated writeTo, v2/LogOutter.java:518-546): header, type 1, term 2, index 3, data 6,
    checksum 7.  Returns (records u8[], record offsets u64[N+1])."""
    n = len(offsets) - 1
    parts = []
    roff = np.zeros(n + 1, np.uint64)
    pos = 0
    for i in range(n):
        ln = int(offsets[i + 1] - offsets[i])
        head = (V2_HEADER + b"\x08" + pb_varint(int(etype[i])) + b"\x10" + pb_varint(int(term[i]))
                + b"\x18" + pb_varint(int(index[i])) + b"\x32" + pb_varint(ln))
        tail = b"\x38" + pb_varint(int(checksum[i]))
        parts += [head, payload[offsets[i]:offsets[i + 1]].tobytes(), tail]
        pos += len(head) + ln + len(tail)
        roff[i + 1] = pos
    return np.frombuffer(b"".join(parts), np.uint8), roff


def quorum_epoch_series(cfg: str, K: int, groups: int | None = None, step: int = 16,
                        seed: int | None = None):
    """K successive epochs of one group batch: epoch 0 = quorum_batch(cfg); each later epoch
    appends `step` entries per group (lastAppended grows) and every follower's match index
    moves forward by 0..2*step, capped at lastAppended (acks stay contiguous, Replicator.java:
    1387-1401).  Returns dict(match[K][P][G], last_appended[K][G], pending_index,
    last_committed, conf) -- the state before epoch 0 plus per-epoch snapshots."""
    b = quorum_batch(cfg, groups=groups, seed=seed)
    P, G = b["match"].shape
    match = np.empty((K, P, G), np.int64)
    la = np.empty((K, G), np.int64)
    match[0], la[0] = b["match"], b["last_appended"]
    s = (SEED_BASE ^ 0xE0) if seed is None else seed ^ 0xE0
    for k in range(1, K):
        la[k] = la[k - 1] + step
        adv = (splitmix64(s + k, P * G).reshape(P, G) % np.uint64(2 * step + 1)).astype(np.int64)
        match[k] = np.minimum(match[k - 1] + adv, la[k])
        match[k, 0] = la[k]  # the leader's own stable ack
    return dict(match=match, last_appended=la, pending_index=b["pending_index"],
                last_committed=b["last_committed"], conf=b["conf"])


def host_series(cfg: str, K: int, groups: int | None = None, joint_frac: float = 0.01,
                active: float = 1.0, step: int = 16, seed: int | None = None):
    """An epoch series for the host-mirror driver (jraft_amd.drive): quorum_epoch_series plus
    (a) a conf change inside the pending window of `joint_frac` of the groups -- entries from
    switch_at[g] on are under conf_b = the stable new conf (NodeImpl's STAGE_STABLE entry after
    the joint one), the earlier ones under conf_a = the group's joint conf -- and (b) per
    epoch only an `active` fraction of the groups gets new entries and acks.  Also returns the
    run table (run_off / run_start / run_conf, conf flagged CONF_RUNS) of the same batch for
    the stateless kernels and the oracle."""
    from ._lib import CONF_RUNS
    s = quorum_epoch_series(cfg, K, groups=groups, step=step, seed=seed)
    P, G = s["match"].shape[1], s["match"].shape[2]
    sd = (SEED_BASE ^ 0xC0) if seed is None else seed ^ 0xC0
    r = splitmix64(sd, G, 1)
    joint = (r % np.uint64(1_000_000)).astype(np.float64) / 1e6 < joint_frac
    pend = s["last_appended"][0] - s["pending_index"] + 1
    off = 1 + (splitmix64(sd, G, 2) % np.maximum(pend - 1, 1).astype(np.uint64)).astype(np.int64)
    switch_at = np.where(joint, s["pending_index"] + off, 0).astype(np.int64)
    conf_a = s["conf"].astype(np.uint64)
    conf_b = np.full(G, conf_word((1 << P) - 1), np.uint64)
    if active < 1.0:
        la, m = s["last_appended"], s["match"]
        for k in range(1, K):
            idle = (splitmix64(sd + k, G, 3) % np.uint64(1_000_000)).astype(np.float64) / 1e6 >= active
            # held at epoch k-1's values; later epochs stay non-decreasing (each was drawn
            # at or above the original epoch k)
            la[k, idle] = la[k - 1, idle]
            m[k][:, idle] = m[k - 1][:, idle]
    nruns = np.where(joint, 2, 1)
    run_off = np.zeros(G + 1, np.uint32)
    run_off[1:] = np.cumsum(nruns)
    run_start = np.zeros(int(run_off[-1]), np.int64)
    run_conf = np.zeros(int(run_off[-1]), np.uint64)
    run_start[run_off[:-1]] = 0
    run_conf[run_off[:-1]] = conf_a
    jr = np.nonzero(joint)[0]
    run_start[run_off[jr] + 1] = switch_at[jr]
    run_conf[run_off[jr] + 1] = conf_b[jr]
    conf = np.where(joint, conf_a | np.uint64(CONF_RUNS), conf_a).astype(np.uint64)
    return dict(match=s["match"], last_appended=s["last_appended"], pending_index=s["pending_index"],
                last_committed=s["last_committed"], conf_a=conf_a, conf_b=conf_b,
                switch_at=switch_at, conf=conf, run_off=run_off, run_start=run_start,
                run_conf=run_conf)
