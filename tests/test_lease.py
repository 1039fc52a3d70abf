"""Leader lease / alive-quorum check: the oracle restatement of
NodeImpl.checkDeadNodes0 / handleStepDownTimeout (NodeImpl.java:1970-2016) on CPU, and the
GPU batch (jrq_lease_check) against it."""
import numpy as np
import pytest

from jraft_amd import conf_word

I64MAX = (1 << 63) - 1


def random_lease_batch(seed, G, P):
    rng = np.random.default_rng(seed)
    now = 10_000_000
    timeout = 900  # ms (electionTimeoutMs 1000 * leaderLeaseTimeRatio 90 %)
    ts = now - rng.integers(0, 2 * timeout, (P, G)).astype(np.int64)
    ts[:, rng.random(G) < 0.05] = 0  # never contacted
    masks = []
    for _ in range(G):
        nm = int(rng.integers(1, 1 << P))
        om = int(rng.integers(1, 1 << P)) if rng.random() < 0.3 else 0
        masks.append(conf_word(nm, om))
    conf = np.array(masks, np.uint64)
    self_slot = rng.integers(0, P, G).astype(np.uint8)
    lead = rng.integers(0, now, G).astype(np.int64)
    return ts, conf, self_slot, now, timeout, lead


def test_reference_semantics(oracle):
    """3 peers, leader slot 0: one follower fresh -> quorum 2 alive, lease from its timestamp;
    both followers stale -> step down; a lone leader keeps lease start Long.MAX_VALUE."""
    now, to = 5000, 900
    ts = np.array([[0, 0, 0], [4500, 3000, 4950], [3000, 3000, 4000]], np.int64)  # [P][G]
    conf = np.array([conf_word(0b111)] * 2 + [conf_word(0b001)], np.uint64)
    ok, lead, dead = oracle.lease_check(ts, conf, [0, 0, 0], now, to, [7, 7, 7])
    assert list(ok) == [3, 2, 3]
    assert lead[0] == 4500 and lead[1] == 7 and lead[2] == I64MAX
    assert list(dead) == [0b100, 0b110, 0]
    # boundary: now - ts == timeout is alive (<=)
    ok, lead, _ = oracle.lease_check(np.array([[0], [4100], [0]], np.int64),
                                     np.array([conf_word(0b011)], np.uint64), [0], now, to, [1])
    assert ok[0] == 3 and lead[0] == 4100


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 3, 5, 8, 16])
def test_gpu_matches_oracle(engine, oracle, P):
    ts, conf, self_slot, now, to, lead = random_lease_batch(P, 5000, P)
    e = oracle.lease_check(ts, conf, self_slot, now, to, lead)
    g = engine.lease_check(ts, conf, self_slot, now, to, lead)
    for a, b in zip(g, e):
        np.testing.assert_array_equal(a, b)
