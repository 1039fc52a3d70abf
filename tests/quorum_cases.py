"""Random group batches for quorum parity tests (inputs only; the oracle decides the answers).

Covers what the reference's BallotBox handles: stable confs, joint consensus
(old + new, ConfigurationCtx STAGE_JOINT, NodeImpl.java:457-487), conf runs inside
the pending window (conf entries, NodeImpl.java:2065-2086), even-size removal
(the non-monotone commit of BallotBox.java:124-129), empty confs, old conf present
but empty, not-leader groups (pendingIndex 0) and out-of-range acks (AIOOBE).
"""
import numpy as np

from jraft_amd import conf_word


def random_mask(rng, P, k):
    return int(sum(1 << int(s) for s in rng.choice(P, size=k, replace=False)))


def random_conf(rng, P, allow_empty=True):
    """A conf word: new conf of 1..P peers (rarely empty), optional old conf."""
    kind = rng.random()
    nn = 0 if (allow_empty and rng.random() < 0.03) else int(rng.integers(1, P + 1))
    new = random_mask(rng, P, nn) if nn else 0
    if kind < 0.5:
        return conf_word(new)  # stable: oldConf == null
    if kind < 0.53:
        return conf_word(new, 0, old_present=True)  # old conf present but empty
    no = int(rng.integers(1, P + 1))
    return conf_word(new, random_mask(rng, P, no))


def random_batch(seed, G, P, pend_max=64, run_prob=0.5, edge=True, max_runs=4):
    rng = np.random.default_rng(seed)
    pi = rng.integers(1, 1 << 20, G).astype(np.int64)
    npend = rng.integers(0, pend_max + 1, G)
    la = pi + npend - 1
    lc = pi - 1 - rng.integers(0, 3, G)
    lc = np.maximum(lc, 0)
    match = np.empty((P, G), np.int64)
    for p in range(P):
        # mostly inside [pi-1, la], sometimes lagging far behind, sometimes 0
        m = pi - 1 + rng.integers(0, npend + 1)
        lag = rng.random(G) < 0.1
        m[lag] = np.maximum(0, pi[lag] - 1 - rng.integers(0, 100, lag.sum()))
        match[p] = m
    conf = np.array([random_conf(rng, P) for _ in range(G)], dtype=np.uint64)
    if edge:
        nl = rng.random(G) < 0.03  # not leader
        pi[nl] = 0
        oor = rng.random(G) < 0.03  # an ack past lastAppended
        rows = np.where(oor)[0]
        match[rng.integers(0, P, len(rows)), rows] = la[rows] + 1 + rng.integers(0, 5, len(rows))
    # conf runs: 2..max_runs runs per flagged group over the pending window
    run_off = [0]
    run_start, run_conf = [], []
    use_runs = rng.random(G) < run_prob
    for g in range(G):
        nr = int(rng.integers(2, max_runs + 1)) if use_runs[g] else 1
        starts = sorted(set(int(x) for x in rng.integers(pi[g], max(pi[g] + 1, la[g] + 2), nr - 1)))
        run_start.append(int(pi[g]) - int(rng.integers(0, 5)))  # first start <= pendingIndex
        run_conf.append(int(conf[g]))
        for s in starts:
            run_start.append(s)
            run_conf.append(random_conf(rng, P))
        run_off.append(len(run_start))
    return dict(match=match, pending_index=pi, last_appended=la, last_committed=lc, conf=conf,
                run_off=np.array(run_off, np.uint32), run_start=np.array(run_start, np.int64),
                run_conf=np.array(run_conf, np.uint64))


def even_removal_batch():
    """4 peers -> 3 peers: entries under the old 4-peer conf need 3 acks, the conf entry and
    later ones (new 3-peer conf) need 2: the later entry commits first and takes the earlier
    ones with it (BallotBox.java:124-129)."""
    P = 4
    pi = np.array([10], np.int64)
    la = np.array([15], np.int64)
    lc = np.array([9], np.int64)
    match = np.array([[15], [15], [11], [11]], np.int64)  # peers 0,1 acked all; 2,3 only to 11
    run_off = np.array([0, 2], np.uint32)
    run_start = np.array([10, 13], np.int64)  # [10,12] old conf 4 peers, [13,15] conf {0,1,2}
    run_conf = np.array([conf_word(0b1111), conf_word(0b0111)], np.uint64)
    return dict(match=match, pending_index=pi, last_appended=la, last_committed=lc,
                conf=run_conf[:1].copy(), run_off=run_off, run_start=run_start, run_conf=run_conf)


def flag_runs(b):
    """conf words flagged CONF_RUNS for the groups with more than one run (as the host variant
    derives them), for calling the *_dev entry points with a run table."""
    from jraft_amd import CONF_RUNS
    ro = b["run_off"]
    cnt = ro[1:] - ro[:-1]
    one = b["run_conf"][np.minimum(ro[:-1], len(b["run_conf"]) - 1)] if len(b["run_conf"]) else b["conf"]
    conf = np.where(cnt == 1, one & np.uint64(~CONF_RUNS & (2**64 - 1)),
                    b["conf"] | np.uint64(CONF_RUNS))
    return conf.astype(np.uint64)


def random_series(seed, G, P, K, run_prob=0.3, step=8):
    """K successive epochs of one group batch with fixed conf runs: epoch k's match snapshot and
    lastAppended (both non-decreasing over k), the state before epoch 0 and the run table.
    Some groups are not the leader, some acks run past lastAppended."""
    b = random_batch(seed, G, P, pend_max=32, run_prob=run_prob)
    rng = np.random.default_rng(seed + 7)
    la = np.empty((K, G), np.int64)
    match = np.empty((K, P, G), np.int64)
    la[0] = b["last_appended"]
    match[0] = b["match"]
    for k in range(1, K):
        la[k] = la[k - 1] + rng.integers(0, step + 1, G)
        adv = rng.integers(0, 2 * step + 1, (P, G))
        stay = rng.random((P, G)) < 0.3
        match[k] = np.where(stay, match[k - 1], np.minimum(np.maximum(match[k - 1], 0) + adv, la[k]))
        oor = rng.random(G) < 0.02
        rows = np.where(oor)[0]
        match[k, rng.integers(0, P, len(rows)), rows] = la[k, rows] + 1
    return dict(match=match, last_appended=la, pending_index=b["pending_index"],
                last_committed=b["last_committed"], conf=b["conf"], run_off=b["run_off"],
                run_start=b["run_start"], run_conf=b["run_conf"])


def series_replay(oracle, s, chunk=5):
    """Expected committed/status of every epoch: K sequential oracle replays, the state carried
    as BallotBox carries it (commit -> lastCommittedIndex, pendingIndex = commit + 1)."""
    K = s["match"].shape[0]
    pi = s["pending_index"].copy()
    lc = s["last_committed"].copy()
    outs, sts = [], []
    for k in range(K):
        ce, se, _ = oracle.quorum_epoch_replay(s["match"][k], pi, s["last_appended"][k], lc,
                                               s["conf"], s.get("run_off"), s.get("run_start"),
                                               s.get("run_conf"), chunk=chunk)
        pi = np.where((pi != 0) & (ce > lc), ce + 1, pi)
        lc = ce
        outs.append(ce)
        sts.append(se)
    return np.stack(outs), np.stack(sts)
