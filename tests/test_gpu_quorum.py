"""GPU parity: libjrq quorum epoch kernel vs replaying the same acks through the
oracle's Java-faithful BallotBox (jraft-core/.../core/BallotBox.java:96-139,
entity/Ballot.java:63-140).  Bit-exact on committed index and status flags.
"""
import numpy as np
import pytest

from jraft_amd import ST_NOT_LEADER, conf_word
from jraft_amd import workloads as W
from quorum_cases import even_removal_batch, random_batch
from devio import to_dev, host_np

pytestmark = pytest.mark.gpu


def _replay(oracle, b, runs=True, chunk=7):
    kw = dict(run_off=b["run_off"], run_start=b["run_start"], run_conf=b["run_conf"]) if runs else {}
    c, s, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                         b["last_committed"], b["conf"], chunk=chunk, **kw)
    return c, s


def _gpu(engine, b, runs=True):
    kw = dict(run_off=b["run_off"], run_start=b["run_start"], run_conf=b["run_conf"]) if runs else {}
    return engine.quorum_epoch(b["match"], b["pending_index"], b["last_appended"],
                               b["last_committed"], b["conf"], **kw)


def test_ballot_box_test_scenario(engine):
    """BallotBoxTest.testCommitAt: conf {8081,8082,8083}, oldConf {8081}; acks from 8081 then
    8082 on entry 1 commit index 1 (jraft-core/src/test/.../core/BallotBoxTest.java:109-137)."""
    b = dict(match=np.array([[1], [1], [0]], np.int64), pending_index=np.array([1], np.int64),
             last_appended=np.array([1], np.int64), last_committed=np.array([0], np.int64),
             conf=np.array([conf_word(0b111, 0b001)], np.uint64))
    c, s = _gpu(engine, b, runs=False)
    assert c[0] == 1 and s[0] == 0
    b["match"] = np.array([[1], [0], [0]], np.int64)  # only 8081: new quorum 2 not reached
    c, s = _gpu(engine, b, runs=False)
    assert c[0] == 0


def test_not_leader_returns_state(engine):
    b = dict(match=np.array([[5], [5], [5]], np.int64), pending_index=np.array([0], np.int64),
             last_appended=np.array([5], np.int64), last_committed=np.array([3], np.int64),
             conf=np.array([conf_word(0b111)], np.uint64))
    c, s = _gpu(engine, b, runs=False)
    assert c[0] == 3 and s[0] == ST_NOT_LEADER


def test_even_size_removal(engine, oracle):
    b = even_removal_batch()
    c, s = _gpu(engine, b)
    ce, se = _replay(oracle, b)
    assert c[0] == ce[0] == 15
    assert s[0] == se[0]


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 7, 8, 16])
def test_random_batches(engine, oracle, P):
    b = random_batch(100 + P, 3000, P)
    c, s = _gpu(engine, b)
    ce, se = _replay(oracle, b)
    np.testing.assert_array_equal(c, ce)
    np.testing.assert_array_equal(s, se)


@pytest.mark.parametrize("P", [3, 5])
def test_random_batches_single_run(engine, oracle, P):
    b = random_batch(200 + P, 3000, P, run_prob=0.0)
    c, s = _gpu(engine, b, runs=False)
    ce, se = _replay(oracle, b, runs=False)
    np.testing.assert_array_equal(c, ce)
    np.testing.assert_array_equal(s, se)


@pytest.mark.parametrize("G", [1, 2, 3, 2999, 3001])
def test_pair_and_scalar_paths(engine, oracle, G):
    """Even G with aligned arrays takes the two-groups-per-lane kernel, odd G the scalar one;
    a device batch whose match rows have an odd stride is forced onto the scalar kernel."""
    import torch
    b = random_batch(300 + G, G, 5, run_prob=0.0)
    ce, se = _replay(oracle, b, runs=False)
    c, s = _gpu(engine, b, runs=False)
    np.testing.assert_array_equal(c, ce)
    np.testing.assert_array_equal(s, se)
    dev = torch.device("cuda:0")
    wide = np.zeros((5, G + 1), np.int64)
    wide[:, :G] = b["match"]
    tm = to_dev(wide, dev)[:, :G]  # row stride G + 1
    t = {k: to_dev(v.view(np.int64) if v.dtype == np.uint64 else v, dev)
         for k, v in b.items() if k in ("pending_index", "last_appended", "last_committed", "conf")}
    out = torch.empty(G, dtype=torch.int64, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_dev(tm, t["pending_index"], t["last_appended"], t["last_committed"],
                            t["conf"], out, st)
    engine.synchronize()
    np.testing.assert_array_equal(host_np(out), ce)
    np.testing.assert_array_equal(host_np(st), se)


@pytest.mark.parametrize("cfg,G", [("C2", None), ("C3", 2000)])
def test_config_shapes_vs_replay(engine, oracle, cfg, G):
    """C2 at its stated size (all 10k groups x 3 peers, configs[1]) and C3-shaped groups (1k
    pending each, 1024-entry ack chunks as the Replicator sends, RaftOptions.maxEntriesSize =
    1024) replayed through real BallotBoxes."""
    b = W.quorum_batch(cfg, groups=G)
    if G is None:
        assert b["pending_index"].shape[0] == W.CONFIGS[cfg]["groups"] == 10_000
    c, s = _gpu(engine, b, runs=False)
    ce, se = _replay(oracle, b, runs=False, chunk=1024)
    np.testing.assert_array_equal(c, ce)
    np.testing.assert_array_equal(s, se)


def test_full_c3_sampled_and_properties(engine, oracle):
    """Full C3 (1M groups x 5 peers, joint): device-resident path; 4096 random groups are
    replayed through the oracle; every group satisfies lc <= committed <= lastAppended and
    a second epoch on the committed state is idempotent."""
    import torch
    b = W.quorum_batch("C3")
    G = b["pending_index"].shape[0]
    dev = torch.device("cuda:0")
    t = {k: to_dev(v.view(np.int64) if v.dtype == np.uint64 else v, dev)
         for k, v in b.items()}
    committed = torch.empty(G, dtype=torch.int64, device=dev)
    status = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.use_stream(torch.cuda.current_stream().cuda_stream)
    try:
        engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                                t["last_committed"], t["conf"], committed, status)
        again = torch.empty_like(committed)
        st2 = torch.empty_like(status)
        engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"], committed,
                                t["conf"], again, st2)
        torch.cuda.synchronize()
    finally:
        engine.use_stream(None)
    c = host_np(committed)
    assert (c >= b["last_committed"]).all() and (c <= b["last_appended"]).all()
    np.testing.assert_array_equal(host_np(again), c)
    rng = np.random.default_rng(3)
    idx = rng.choice(G, 4096, replace=False)
    sub = {k: (v[:, idx] if k == "match" else v[idx]) for k, v in b.items()}
    ce, se = _replay(oracle, sub, runs=False, chunk=1024)
    np.testing.assert_array_equal(c[idx], ce)
    np.testing.assert_array_equal(host_np(status)[idx], se)


def _series_oracle(s, K):
    import jraft_oracle as O
    pi = s["pending_index"].copy()
    lc = s["last_committed"].copy()
    outs, sts = [], []
    for k in range(K):
        ce, se, _ = O.quorum_epoch_replay(s["match"][k], pi, s["last_appended"][k], lc, s["conf"],
                                          chunk=1024)
        pi = np.where((pi != 0) & (ce > lc), ce + 1, pi)
        lc = ce
        outs.append(ce)
        sts.append(se)
    return np.stack(outs), np.stack(sts)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,G,K", [("C2", 1000, 7), ("C3", 3000, 9), ("C2", 1, 1),
                                     ("C2", 10_000, 64), ("C2", 10_000, 256), ("C3", 3000, 300),
                                     ("C2", 33, 129)])
def test_gpu_quorum_epochs_series_vs_oracle(engine, cfg, G, K):
    """K epochs in one launch == K sequential BallotBox replays with carried state."""
    import torch

    from jraft_amd import workloads as W
    s = W.quorum_epoch_series(cfg, K, groups=G)
    s["pending_index"][::97] = 0  # some groups are not the leader
    dev = torch.device("cuda", 0)
    t = {k: to_dev(np.ascontiguousarray(v.view(np.int64) if v.dtype == np.uint64 else v), dev)
         for k, v in s.items()}
    c = torch.empty((K, G), dtype=torch.int64, device=dev)
    st = torch.empty((K, G), dtype=torch.uint8, device=dev)
    engine.quorum_epochs_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], c, st)
    engine.synchronize()
    ce, se = _series_oracle(s, K)
    assert np.array_equal(host_np(c), ce)
    assert np.array_equal(host_np(st), se)
    if K > 1:
        assert (ce[-1] > ce[0]).any()  # commits actually move across epochs


@pytest.mark.gpu
def test_gpu_quorum_epochs_relaunch_sequence(engine):
    """jrq_quorum_epochs_dev over a sequence of launch shapes on one engine: both chunk depths
    (C = 4 below 192 epochs per launch, C = 8 from there), batches of 313 to 3750 tiles of 16
    groups (the larger ones with many super-chunks per workgroup), and repeated launches of one
    batch that must give identical results.  Groups are checked against the oracle on a sample
    of columns (each group's epochs are independent of the others')."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    first = {}
    for rep, (G, K) in enumerate([(10_000, 256), (60_000, 512), (500, 100), (10_000, 256),
                                  (60_000, 512), (10_000, 256)]):
        s = W.quorum_epoch_series("C2", K, groups=G)
        s["pending_index"][::89] = 0
        t = {k: to_dev(np.ascontiguousarray(v.view(np.int64) if v.dtype == np.uint64 else v), dev)
             for k, v in s.items()}
        c = torch.empty((K, G), dtype=torch.int64, device=dev)
        st = torch.empty((K, G), dtype=torch.uint8, device=dev)
        engine.quorum_epochs_dev(t["match"], t["pending_index"], t["last_appended"],
                                 t["last_committed"], t["conf"], c, st)
        engine.synchronize()
        got_c, got_s = host_np(c), host_np(st)
        if (G, K) in first:
            assert np.array_equal(got_c, first[(G, K)][0]) and np.array_equal(got_s, first[(G, K)][1])
            continue
        first[(G, K)] = (got_c, got_s)
        sub = np.sort(rng.choice(G, min(G, 96), replace=False))
        ss = {"match": s["match"][:, :, sub], "last_appended": s["last_appended"][:, sub],
              "pending_index": s["pending_index"][sub], "last_committed": s["last_committed"][sub],
              "conf": s["conf"][sub]}
        ce, se = _series_oracle(ss, K)
        assert np.array_equal(got_c[:, sub], ce), (G, K)
        assert np.array_equal(got_s[:, sub], se), (G, K)


def _to_dev(b, keys):
    import torch
    dev = torch.device("cuda:0")
    return {k: to_dev(np.ascontiguousarray(b[k].view(np.int64) if b[k].dtype == np.uint64
                                                     else b[k]), dev) for k in keys}


@pytest.mark.parametrize("P,run_prob,max_runs,G", [(5, 0.01, 4, 4096), (3, 0.3, 4, 4096),
                                                   (8, 0.05, 4, 4096), (5, 0.9, 9, 4098),
                                                   (16, 0.5, 6, 1030), (1, 0.2, 3, 2048)])
def test_dev_fast_path_with_flagged_runs(engine, oracle, P, run_prob, max_runs, G):
    """Device batch with aligned arrays (pair kernel) where only JRQ_CONF_RUNS groups walk the
    run table: a conf-changing group no longer demotes the launch, and every group -- flagged
    or not -- matches the replay through real BallotBoxes.  Each wave walks its own flagged
    groups, four lanes per group: 90 % flagged puts more than the 16 LDS hand-off slots'
    worth in a wave (the reload path), up to 9 runs loops a lane over runs r, r + 4, r + 8."""
    import torch
    from quorum_cases import flag_runs
    b = random_batch(500 + P, G, P, run_prob=run_prob, max_runs=max_runs)
    b["conf"] = flag_runs(b)
    ce, se = _replay(oracle, b)
    t = _to_dev(b, ["match", "pending_index", "last_appended", "last_committed", "conf",
                    "run_off", "run_start", "run_conf"])
    out = torch.empty(G, dtype=torch.int64, device="cuda:0")
    st = torch.empty(G, dtype=torch.uint8, device="cuda:0")
    engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                            t["last_committed"], t["conf"], out, st, run_off=t["run_off"],
                            run_start=t["run_start"], run_conf=t["run_conf"])
    engine.synchronize()
    np.testing.assert_array_equal(host_np(out), ce)
    np.testing.assert_array_equal(host_np(st), se)


@pytest.mark.parametrize("P,run_prob,max_runs,G", [(5, 0.01, 4, 4096), (3, 0.3, 4, 4097),
                                                   (5, 0.9, 9, 1030), (16, 0.5, 6, 515),
                                                   (1, 0.2, 3, 2), (8, 0.0, 1, 300)])
def test_tiles_entry_point_vs_replay(engine, oracle, P, run_prob, max_runs, G):
    """jrq_quorum_epoch_tiles_dev: the same batches in the resident table's tile layout
    (W.to_tiles: 256-group tiles, G not a multiple of 256, odd G, more flagged groups per wave
    than hand-off slots) decide exactly as the replay through real BallotBoxes."""
    import torch
    from quorum_cases import flag_runs
    b = random_batch(700 + P, G, P, run_prob=run_prob, max_runs=max_runs)
    b["conf"] = flag_runs(b)
    ce, se = _replay(oracle, b)
    dev = torch.device("cuda:0")
    tiles = to_dev(W.to_tiles(b["match"], b["pending_index"], b["last_appended"],
                                        b["last_committed"], b["conf"]), dev)
    t = _to_dev(b, ["run_off", "run_start", "run_conf"])
    out = torch.empty(G, dtype=torch.int64, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_tiles_launcher(tiles, P, G, out, st, t["run_off"], t["run_start"],
                                       t["run_conf"])()
    engine.synchronize()
    np.testing.assert_array_equal(host_np(out), ce)
    np.testing.assert_array_equal(host_np(st), se)


def test_tiles_entry_point_full_c3(engine):
    """C3 at its full 1M groups through the tile layout: identical to the rows entry point
    (itself checked against the oracle on C3 by test_full_c3_sampled_and_properties)."""
    import torch
    b = W.quorum_batch("C3")
    P, G = b["match"].shape[0], b["match"].shape[1]
    dev = torch.device("cuda:0")
    t = _to_dev(b, ["match", "pending_index", "last_appended", "last_committed", "conf"])
    o1 = torch.empty(G, dtype=torch.int64, device=dev)
    s1 = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                            t["last_committed"], t["conf"], o1, s1)
    tiles = to_dev(W.to_tiles(b["match"], b["pending_index"], b["last_appended"],
                                        b["last_committed"], b["conf"]), dev)
    o2 = torch.empty(G, dtype=torch.int64, device=dev)
    s2 = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_tiles_launcher(tiles, P, G, o2, s2)()
    engine.synchronize()
    assert torch.equal(o1, o2) and torch.equal(s1, s2)


def _series_tiles(s, K):
    """Every epoch of series `s` in the tile layout, one row per epoch (W.to_tiles)."""
    return np.stack([W.to_tiles(s["match"][k], s["pending_index"], s["last_appended"][k],
                                s["last_committed"], s["conf"]) for k in range(K)])


@pytest.mark.parametrize("P,G,K,runs", [(3, 1000, 9, False), (5, 778, 12, True), (2, 64, 1, False),
                                        (5, 777, 1, True), (3, 130, 40, True)])
def test_gpu_quorum_epochs_tiles_vs_replay(engine, oracle, P, G, K, runs):
    """jrq_quorum_epochs_tiles_dev: K epochs with each epoch's inputs in the tile layout ==
    K sequential BallotBox replays with carried state (conf runs and flagged groups included,
    G off the tile grid, odd G for one epoch)."""
    import torch
    from quorum_cases import flag_runs, random_series, series_replay
    s = random_series(1900 + K, G, P, K)
    if runs:
        s["conf"] = flag_runs(s)
    else:
        s["conf"] = s["conf"] & ~np.uint64(1 << 63)
        s["run_off"] = None
    ce, se = series_replay(oracle, s) if runs else _series_oracle(
        {k: v for k, v in s.items() if k != "run_off"}, K)
    dev = torch.device("cuda:0")
    tiles = to_dev(_series_tiles(s, K), dev)
    rt = _to_dev(s, ["run_off", "run_start", "run_conf"]) if runs else {}
    c = torch.empty((K, G), dtype=torch.int64, device=dev)
    st = torch.empty((K, G), dtype=torch.uint8, device=dev)
    engine.quorum_epochs_tiles_launcher(tiles, P, G, c, st, rt.get("run_off"), rt.get("run_start"),
                                        rt.get("run_conf"))()
    engine.synchronize()
    np.testing.assert_array_equal(host_np(c), ce)
    np.testing.assert_array_equal(host_np(st), se)


def test_gpu_quorum_epochs_tiles_full_c3(engine):
    """C3 at its full 1M groups, 4 epochs per launch, tiles against the rows entry point (itself
    checked against the oracle on large batches above); odd G with K > 1 is refused (its
    committed rows would lose the 16-B alignment of the pair stores)."""
    import torch
    from jraft_amd import JrqError
    K = 4
    s = W.quorum_epoch_series("C3", K)
    G = s["pending_index"].shape[0]
    dev = torch.device("cuda:0")
    d = {k: to_dev(np.ascontiguousarray(v.view(np.int64) if v.dtype == np.uint64 else v), dev)
         for k, v in s.items()}
    c1 = torch.empty((K, G), dtype=torch.int64, device=dev)
    s1 = torch.empty((K, G), dtype=torch.uint8, device=dev)
    engine.quorum_epochs_dev(d["match"], d["pending_index"], d["last_appended"], d["last_committed"],
                             d["conf"], c1, s1)
    tiles = to_dev(_series_tiles(s, K), dev)
    c2 = torch.empty((K, G), dtype=torch.int64, device=dev)
    s2 = torch.empty((K, G), dtype=torch.uint8, device=dev)
    engine.quorum_epochs_tiles_launcher(tiles, 5, G, c2, s2)()
    engine.synchronize()
    assert torch.equal(c1, c2) and torch.equal(s1, s2)
    assert (c1[-1] > c1[0]).any()
    with pytest.raises(JrqError):
        engine.quorum_epochs_tiles_launcher(tiles, 5, G - 1, c2, s2)()


@pytest.mark.parametrize("P,G,K", [(3, 1000, 9), (5, 777, 40), (2, 64, 1), (3, 130, 200),
                                   (16, 300, 70), (9, 500, 200), (1, 100, 300), (16, 40, 193)])
def test_gpu_quorum_epochs_with_runs(engine, oracle, P, G, K):
    """K epochs in one launch with conf runs and flagged groups == K sequential replays."""
    import torch
    from quorum_cases import flag_runs, random_series, series_replay
    s = random_series(900 + K, G, P, K)
    s["conf"] = flag_runs(s)
    ce, se = series_replay(oracle, s)
    t = _to_dev(s, list(s.keys()))
    c = torch.empty((K, G), dtype=torch.int64, device="cuda:0")
    st = torch.empty((K, G), dtype=torch.uint8, device="cuda:0")
    engine.quorum_epochs_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], c, st, run_off=t["run_off"],
                             run_start=t["run_start"], run_conf=t["run_conf"])
    engine.synchronize()
    np.testing.assert_array_equal(host_np(c), ce)
    np.testing.assert_array_equal(host_np(st), se)


def test_host_variant_rejects_bad_run_csr(engine):
    """jrq_quorum_epoch checks the run table CSR on the host before staging it (run_off[0] =
    0, monotone, run_off[G] = the number of runs): a bad one is JRQ_E_INVALID, not a device
    read past the staged runs."""
    from jraft_amd import JrqError
    b = random_batch(5, 64, 3, run_prob=0.5)
    args = (b["match"], b["pending_index"], b["last_appended"], b["last_committed"], b["conf"])
    bad = b["run_off"].copy()
    bad[10], bad[11] = bad[11] + 1, bad[10]          # not monotone
    with pytest.raises(JrqError):
        engine.quorum_epoch(*args, run_off=bad, run_start=b["run_start"], run_conf=b["run_conf"])
    short = b["run_off"].copy()
    short[-1] += 3                                   # past the runs given
    with pytest.raises(JrqError):
        engine.quorum_epoch(*args, run_off=short, run_start=b["run_start"], run_conf=b["run_conf"])
    c, _ = engine.quorum_epoch(*args, run_off=b["run_off"], run_start=b["run_start"],
                               run_conf=b["run_conf"])
    assert c.shape == (64,)



def _decide_single_ref(pi, la, lc, cw, m):
    """The single-conf decision in plain int64 arithmetic (quorum_core.h decide_single; the
    formulation test_quorum_model.py checks against BallotBox replays): committed, status."""
    from jraft_amd import ST_EMPTY_CONF, ST_NOT_LEADER, ST_OUT_OF_RANGE
    P = len(m)
    if pi == 0:
        return lc, ST_NOT_LEADER
    st = 0
    v = []
    for p in range(P):
        if m[p] > la:
            st |= ST_OUT_OF_RANGE
            v.append(None)
        else:
            v.append(int(m[p]))
    if (cw & 0xFFFF) == 0 and la >= pi:
        st |= ST_EMPTY_CONF

    def kth(mask, q):
        if q == 0:
            return float("inf")
        vals = sorted((x for p, x in enumerate(v) if (mask >> p) & 1 and x is not None), reverse=True)
        return vals[q - 1] if q <= len(vals) else float("-inf")
    cand = min(kth(cw & 0xFFFF, (cw >> 32) & 0xFF), kth((cw >> 16) & 0xFFFF, (cw >> 40) & 0xFF), la)
    return (int(cand) if cand >= pi and cand > lc else lc), st


def test_pair_kernel_32bit_domain_edges(engine):
    """The pair kernel decides in 32-bit arithmetic relative to pendingIndex (decide_single_rel)
    and sends groups outside that domain -- negative or huge pendingIndex, windows of 2^32 - 1
    entries and more -- through a 64-bit second pass.  Edge groups of every kind, mixed into
    waves with ordinary ones, against the decision in Python integers."""
    import torch
    rng = np.random.default_rng(77)
    P, G = 5, 4096
    I64 = np.iinfo(np.int64)
    pis = [0, 1, 2, 1 << 31, (1 << 32) + 7, (1 << 62) - 5, 1 << 62, (1 << 62) + 3, -5, I64.max - 10]
    wins = [0, 1, 2, 1000, (1 << 32) - 2, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, 1 << 40]
    pi = np.zeros(G, np.int64)
    la = np.zeros(G, np.int64)
    lc = np.zeros(G, np.int64)
    m = np.zeros((P, G), np.int64)
    conf = np.zeros(G, np.uint64)
    for g in range(G):
        p0 = int(rng.choice(pis)) if rng.random() < 0.6 else int(rng.integers(1, 1 << 40))
        w = int(rng.choice(wins))
        l = max(min(p0 - 1 + w, int(I64.max)), int(I64.min))
        pi[g], la[g] = p0, l
        lc[g] = p0 - 1 - int(rng.integers(0, 3)) if p0 > I64.min + 3 else p0
        for p in range(P):
            c = rng.integers(0, 8)
            val = [p0 - 1, p0, l, l + 1 if l < I64.max else l, p0 + w // 2, -1, int(I64.min),
                   int(I64.max)][c]
            m[p, g] = max(min(val, int(I64.max)), int(I64.min))
        from quorum_cases import random_conf
        conf[g] = random_conf(rng, P)
    ce = np.zeros(G, np.int64)
    se = np.zeros(G, np.uint8)
    for g in range(G):
        c, s = _decide_single_ref(int(pi[g]), int(la[g]), int(lc[g]), int(conf[g]),
                                  [int(x) for x in m[:, g]])
        ce[g], se[g] = c, s
    dev = torch.device("cuda:0")
    t = {k: to_dev(v.view(np.int64) if v.dtype == np.uint64 else v, dev)
         for k, v in dict(match=m, pending_index=pi, last_appended=la, last_committed=lc,
                          conf=conf).items()}
    out = torch.empty(G, dtype=torch.int64, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                            t["last_committed"], t["conf"], out, st)
    engine.synchronize()
    np.testing.assert_array_equal(host_np(out), ce)
    np.testing.assert_array_equal(host_np(st), se)


def _tile_series(s, copies):
    """`copies` back-to-back copies of a random_series batch (its run table's CSR re-based)."""
    n, R = len(s["pending_index"]), len(s["run_start"])
    out = {k: np.concatenate([s[k]] * copies, axis=-1) for k in
           ("match", "last_appended", "pending_index", "last_committed", "conf", "run_start", "run_conf")}
    ro = s["run_off"].astype(np.int64)
    out["run_off"] = np.concatenate([ro[:-1] + c * R for c in range(copies)] + [[copies * R]]).astype(s["run_off"].dtype)
    assert len(out["pending_index"]) == n * copies
    return out


@pytest.mark.parametrize("P,K", [(5, 8), (3, 5)])
def test_gpu_quorum_epochs_large_batch(engine, oracle, P, K):
    """K epochs of a batch large enough for the sequential pair kernel (G >= 2048 per CU, even:
    two groups per lane through every epoch, quorum_epochs_pair_kernel) -- 147 copies of a
    4096-group series with conf runs, flagged groups, non-leaders and out-of-range acks -- equal
    the K sequential BallotBox replays on every copy; G - 1 groups of the same arrays (odd: the
    chunk kernel) agree with it."""
    import torch
    from quorum_cases import flag_runs, random_series, series_replay
    s = random_series(1300 + P, 4096, P, K)
    s["conf"] = flag_runs(s)
    ce, se = series_replay(oracle, s)
    big = _tile_series(s, 147)
    G = len(big["pending_index"])
    assert G % 2 == 0 and G >= 2048 * 256
    t = _to_dev(big, list(big.keys()))
    c = torch.empty((K, G), dtype=torch.int64, device="cuda:0")
    st = torch.empty((K, G), dtype=torch.uint8, device="cuda:0")
    engine.quorum_epochs_dev(t["match"], t["pending_index"], t["last_appended"],
                             t["last_committed"], t["conf"], c, st, run_off=t["run_off"],
                             run_start=t["run_start"], run_conf=t["run_conf"])
    engine.synchronize()
    cg, sg = host_np(c), host_np(st)
    np.testing.assert_array_equal(cg, np.tile(ce, (1, 147)))
    np.testing.assert_array_equal(sg, np.tile(se, (1, 147)))
    # the chunk kernel on G - 1 groups of the same arrays (rows keep their strides)
    G1 = G - 1
    c1 = torch.empty((K, G1), dtype=torch.int64, device="cuda:0")
    s1 = torch.empty((K, G1), dtype=torch.uint8, device="cuda:0")
    engine.quorum_epochs_dev(t["match"][:, :, :G1], t["pending_index"][:G1], t["last_appended"][:, :G1],
                             t["last_committed"][:G1], t["conf"][:G1], c1, s1, run_off=t["run_off"][:G1 + 1],
                             run_start=t["run_start"], run_conf=t["run_conf"])
    engine.synchronize()
    np.testing.assert_array_equal(host_np(c1), cg[:, :G1])
    np.testing.assert_array_equal(host_np(s1), sg[:, :G1])


@pytest.mark.parametrize("P,run_prob,G", [(5, 0.01, 4096), (3, 0.3, 3001), (16, 0.5, 515)])
def test_tiles_host_variant_vs_replay(engine, oracle, P, run_prob, G):
    """jrq_quorum_epoch_tiles (host memory: the JNI binding's one direct buffer of tiles per
    batch) decides exactly as the replay through real BallotBoxes; a bad
    run CSR is refused before any upload."""
    from jraft_amd import JrqError
    from quorum_cases import flag_runs
    b = random_batch(1700 + P, G, P, run_prob=run_prob)
    b["conf"] = flag_runs(b)
    ce, se = _replay(oracle, b)
    tiles = W.to_tiles(b["match"], b["pending_index"], b["last_appended"], b["last_committed"], b["conf"])
    out, st = engine.quorum_epoch_tiles(tiles, P, G, b["run_off"], b["run_start"], b["run_conf"])
    np.testing.assert_array_equal(out, ce)
    np.testing.assert_array_equal(st, se)
    bad = b["run_off"].copy()
    bad[G // 2] = bad[G // 2 + 1] + 1  # not monotone
    with pytest.raises(JrqError):
        engine.quorum_epoch_tiles(tiles, P, G, bad, b["run_start"], b["run_conf"])
