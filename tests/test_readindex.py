"""ReadIndex heartbeat quorum: the ReadOnlySafe round of NodeImpl.readLeader
(NodeImpl.java:1343-1396) decided as ReadIndexHeartbeatResponseClosure.run does
(:1246-1291).  The oracle restatement is checked against an event-by-event Python model of
the closure and the reference's scenarios; the GPU batch (jrq_readindex_quorum) against the
oracle, bit-exact."""
import numpy as np
import pytest

from jraft_amd import conf_word
from devio import to_dev, host_np

PENDING, SUCCESS, FAILURE = 0, 1, 2


class HeartbeatClosure:
    """ReadIndexHeartbeatResponseClosure (NodeImpl.java:1246-1291), one response at a time."""

    def __init__(self, quorum, peers_count):
        self.quorum = quorum
        self.fail_peers_threshold = quorum - 1 if peers_count % 2 == 0 else quorum
        self.ack_success = self.ack_failures = 0
        self.verdict = PENDING

    def run(self, ok):
        if self.verdict != PENDING:  # isDone
            return
        if ok:
            self.ack_success += 1
        else:
            self.ack_failures += 1
        if self.ack_success + 1 >= self.quorum:
            self.verdict = SUCCESS
        elif self.ack_failures >= self.fail_peers_threshold:
            self.verdict = FAILURE


def model(mask, P, self_slot, responses):
    """readLeader: getQuorum (:1321-1327), the fast path, then the responses (slot, ok) in
    arrival order from the peers a heartbeat went to."""
    peers = [s for s in range(16) if mask >> s & 1]
    quorum = len(peers) // 2 + 1 if peers else 0
    if quorum <= 1:
        return SUCCESS
    c = HeartbeatClosure(quorum, len(peers))
    for slot, ok in responses:
        if slot in peers and slot != self_slot and slot < P:
            c.run(ok)
    return c.verdict


def encode(responses):
    """(slot, ok) in arrival order -> (order word, ok mask)."""
    order, okm = 0, 0
    for pos, (slot, ok) in enumerate(responses, start=1):
        order |= pos << (4 * slot)
        okm |= int(ok) << slot
    return order, okm


def one(oracle, mask, P, self_slot, responses):
    order, okm = encode(responses)
    return int(oracle.readindex_quorum([conf_word(mask)], [self_slot], [order], [okm], P)[0])


def test_reference_scenarios(oracle):
    """3 peers, leader slot 0 (quorum 2, failure threshold 2): one success answers; one failure
    waits, two fail.  4 peers (quorum 3, threshold 2 for an even count).  One peer / empty
    conf: the fast path.  Leader outside its conf (3 peers, three heartbeats): the arrival
    order decides."""
    assert one(oracle, 0b111, 3, 0, []) == PENDING
    assert one(oracle, 0b111, 3, 0, [(1, True)]) == SUCCESS
    assert one(oracle, 0b111, 3, 0, [(1, False)]) == PENDING
    assert one(oracle, 0b111, 3, 0, [(1, False), (2, False)]) == FAILURE
    assert one(oracle, 0b111, 3, 0, [(1, False), (2, True)]) == SUCCESS
    assert one(oracle, 0b1111, 4, 0, [(1, True)]) == PENDING
    assert one(oracle, 0b1111, 4, 0, [(1, True), (3, True)]) == SUCCESS
    assert one(oracle, 0b1111, 4, 0, [(1, False), (2, False)]) == FAILURE
    assert one(oracle, 0b0001, 4, 0, []) == SUCCESS
    assert one(oracle, 0, 4, 0, []) == SUCCESS
    # leader in slot 3, conf {0, 1, 2}: quorum 2, threshold 2; success needs one ok
    assert one(oracle, 0b0111, 4, 3, [(0, False), (1, True), (2, False)]) == SUCCESS
    assert one(oracle, 0b0111, 4, 3, [(0, False), (2, False), (1, True)]) == FAILURE
    # a response from the leader's own slot or a non-member never counts
    assert one(oracle, 0b0111, 4, 0, [(0, True), (3, True)]) == PENDING


def random_rounds(seed, G, P, ties=0.1):
    """Random conf masks (sometimes without the leader), a random subset of the heartbeats
    answered in a random order, some positions tied (the leader's own slot never answers, so
    positions stay within 1..15; non-members may, and are ignored)."""
    rng = np.random.default_rng(seed)
    conf = np.zeros(G, np.uint64)
    self_slot = rng.integers(0, P, G).astype(np.uint8)
    order = np.zeros(G, np.uint64)
    okm = np.zeros(G, np.uint16)
    rounds = []
    for g in range(G):
        mask = int(rng.integers(0, 1 << P))
        if rng.random() < 0.7:
            mask |= 1 << int(self_slot[g])
        conf[g] = conf_word(mask)
        slots = [s for s in range(P) if s != self_slot[g] and rng.random() < 0.7]  # <= 15
        rng.shuffle(slots)
        pos = np.arange(1, len(slots) + 1)
        if len(slots) > 1 and rng.random() < ties:  # two responses at one position
            pos[-1] = pos[-2]
        o, k = 0, 0
        resp = []
        for s, p in zip(slots, pos):
            ok = bool(rng.random() < 0.55)
            o |= int(p) << (4 * s)
            k |= int(ok) << s
            resp.append((int(p), s, ok))
        order[g], okm[g] = o, k
        rounds.append((mask, int(self_slot[g]), [(s, ok) for _, s, ok in sorted(resp)]))
    return conf, self_slot, order, okm, rounds


@pytest.mark.parametrize("P", [1, 3, 5, 16])
def test_oracle_matches_closure_model(oracle, P):
    conf, self_slot, order, okm, rounds = random_rounds(100 + P, 3000, P)
    got = oracle.readindex_quorum(conf, self_slot, order, okm, P)
    want = [model(m, P, s, r) for m, s, r in rounds]
    np.testing.assert_array_equal(got, np.array(want, np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("P,G", [(1, 20000), (2, 20001), (3, 20002), (5, 20003), (8, 3), (16, 20000)])
def test_gpu_matches_oracle(engine, oracle, P, G):
    """The host variant (aligned staging: four groups per lane, G % 4 left over)."""
    conf, self_slot, order, okm, _ = random_rounds(P, G, P, ties=0.2)
    e = oracle.readindex_quorum(conf, self_slot, order, okm, P)
    g = engine.readindex_quorum(conf, self_slot, order, okm, P)
    np.testing.assert_array_equal(g, e)
    assert {0, 1, 2} <= set(np.unique(e)) or P < 3 or G < 100


@pytest.mark.gpu
def test_gpu_unaligned_device_pointers(engine, oracle):
    """Device pointers off the 16-B grid (a slice from element 1): the one-group-per-lane form."""
    import torch
    P, G = 5, 10001
    conf, self_slot, order, okm, _ = random_rounds(11, G + 1, P)
    dev = torch.device("cuda:0")
    tc = to_dev(conf.view(np.int64), dev)
    ts = to_dev(self_slot, dev)
    to = to_dev(order.view(np.int64), dev)
    tk = to_dev(okm.view(np.int16), dev)
    out = torch.zeros(G + 1, dtype=torch.uint8, device=dev)
    engine.readindex_quorum_dev(tc[1:], ts[1:], to[1:], tk[1:], P, out[1:])
    torch.cuda.synchronize()
    got = host_np(out)
    np.testing.assert_array_equal(got[1:], oracle.readindex_quorum(conf[1:], self_slot[1:], order[1:], okm[1:], P))
    assert got[0] == 0


@pytest.mark.gpu
def test_gpu_dev_entry_point_and_rounds_in_steps(engine, oracle):
    """The device entry point over 1M groups (5 peers), and a round's responses fed in two
    steps: a verdict of the first call never changes in the second."""
    import torch
    P, G = 5, 1 << 20
    conf, self_slot, order, okm, _ = random_rounds(7, 4096, P)
    rep = -(-G // 4096)
    conf, self_slot, order, okm = (np.tile(a, rep)[:G] for a in (conf, self_slot, order, okm))
    dev = torch.device("cuda:0")
    # first step: only the responses at positions 1..2
    nib = (order[:, None] >> (4 * np.arange(P, dtype=np.uint64))) & np.uint64(0xF)
    early = np.where((nib >= 1) & (nib <= 2), nib, 0)
    order1 = (early << (4 * np.arange(P, dtype=np.uint64))).sum(axis=1).astype(np.uint64)
    out = torch.empty(G, dtype=torch.uint8, device=dev)
    t = {k: to_dev(v.view(np.int64) if v.dtype == np.uint64 else
                             (v.view(np.int16) if v.dtype == np.uint16 else v), dev)
         for k, v in (("conf", conf), ("self", self_slot), ("o1", order1), ("o", order), ("ok", okm))}
    engine.readindex_quorum_dev(t["conf"], t["self"], t["o1"], t["ok"], P, out)
    torch.cuda.synchronize()
    r1 = host_np(out)
    np.testing.assert_array_equal(r1, oracle.readindex_quorum(conf, self_slot, order1, okm, P))
    engine.readindex_quorum_dev(t["conf"], t["self"], t["o"], t["ok"], P, out)
    torch.cuda.synchronize()
    r2 = host_np(out)
    np.testing.assert_array_equal(r2, oracle.readindex_quorum(conf, self_slot, order, okm, P))
    decided = r1 != PENDING
    np.testing.assert_array_equal(r2[decided], r1[decided])


def _with_stray_slots(P, G, seed):
    """random_rounds plus, for a third of the groups, conf bits at slots >= P (outside the
    batch: ADVICE r04 -- no response can come from them)."""
    conf, self_slot, order, okm, _ = random_rounds(seed, G, P)
    rng = np.random.default_rng(seed + 1)
    stray = rng.random(G) < 1 / 3
    extra = rng.integers(P, 16, G) if P < 16 else np.zeros(G, np.int64)
    conf = np.where(stray, conf | (np.uint64(1) << extra.astype(np.uint64)), conf).astype(np.uint64)
    return conf, self_slot, order, okm, stray


@pytest.mark.parametrize("P", [1, 3, 5, 15])
def test_oracle_conf_beyond_num_peers_is_invalid(oracle, P):
    conf, self_slot, order, okm, stray = _with_stray_slots(P, 2000, 50 + P)
    got = oracle.readindex_quorum(conf, self_slot, order, okm, P)
    assert (got[stray] == 3).all()
    assert (got[~stray] != 3).all()


@pytest.mark.gpu
@pytest.mark.parametrize("P,G", [(3, 20001), (5, 20000), (15, 4099)])
def test_gpu_conf_beyond_num_peers_is_invalid(engine, oracle, P, G):
    conf, self_slot, order, okm, stray = _with_stray_slots(P, G, 60 + P)
    e = oracle.readindex_quorum(conf, self_slot, order, okm, P)
    g = engine.readindex_quorum(conf, self_slot, order, okm, P)
    np.testing.assert_array_equal(g, e)
    assert (g[stray] == 3).all()
