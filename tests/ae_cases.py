"""Random AppendEntries request batches (inputs only) for the follower-verify parity tests."""
import numpy as np


def random_requests(seed, R, max_entries=64, max_len=3000, corrupt_frac=0.02, oracle=None,
                    uniform=None):
    """R requests; entries of random type (incl. UNKNOWN = 0, which consumes no data),
    random data_len, checksums as a leader would stamp them (from the oracle), a few
    flipped so the follower must flag them, a few entries without a checksum.
    uniform=L: every request holds max_entries entries of L bytes, none UNKNOWN (the batch the
    fixed-size data path takes)."""
    rng = np.random.default_rng(seed)
    n_per = rng.integers(0, max_entries + 1, R) if uniform is None else np.full(R, max_entries)
    req_off = np.concatenate([[0], np.cumsum(n_per)]).astype(np.uint32)
    N = int(req_off[-1])
    prev = rng.integers(0, 1 << 40, R).astype(np.int64)
    term = rng.integers(1, 1 << 20, N).astype(np.int64)
    if uniform is None:
        etype = rng.choice([0, 1, 2, 2, 2, 3], N).astype(np.uint8)
        data_len = rng.integers(0, max_len + 1, N).astype(np.int64)
        data_len[rng.random(N) < 0.1] = 0
    else:
        etype = rng.choice([1, 2, 2, 2, 3], N).astype(np.uint8)
        data_len = np.full(N, uniform, np.int64)
    consumed = int(data_len[etype != 0].sum())
    data = rng.integers(0, 256, consumed, dtype=np.uint8)
    peer_xor = (rng.integers(0, 1 << 62, N).astype(np.uint64) * (etype == 3)).astype(np.uint64)
    has = (rng.random(N) < 0.95).astype(np.uint8)
    checksum = np.zeros(N, np.uint64)
    if oracle is not None:
        good, _, _ = oracle.append_entries_verify(req_off, prev, term, etype, data_len, checksum,
                                                  data, has_checksum=np.zeros(N, np.uint8),
                                                  peer_xor=peer_xor)
        checksum = good.copy()
        flip = rng.random(N) < corrupt_frac
        checksum[flip] ^= np.uint64(1) << np.uint64(int(rng.integers(0, 64)))
    return dict(req_off=req_off, prev_log_index=prev, term=term, etype=etype, data_len=data_len,
                checksum=checksum, data=data, has_checksum=has, peer_xor=peer_xor)
