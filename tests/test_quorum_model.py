"""CPU check of the quorum kernel's FORMULATION (quorum.hip) against the oracle replay.

A pure-Python restatement of the kernel's per-group arithmetic (q-th largest match
per conf mask, per-run candidates, max with lastCommitted) is compared with
replaying the same acks through the Java-faithful BallotBox of the oracle.  This
pins the math on CPU; tests/test_gpu_quorum.py pins the device code.
"""
import numpy as np
import pytest

from quorum_cases import even_removal_batch, random_batch

I64MIN = -(1 << 63)
I64MAX = (1 << 63) - 1


def kth(m, mask, q):
    vals = sorted((m[p] for p in range(len(m)) if (mask >> p) & 1), reverse=True)
    return vals[q - 1] if q <= len(vals) else I64MIN


def model(b, runs=True):
    P, G = b["match"].shape
    out, st = [], []
    for g in range(G):
        pi, la, lc = int(b["pending_index"][g]), int(b["last_appended"][g]), int(b["last_committed"][g])
        if pi == 0:
            out.append(lc)
            st.append(1)
            continue
        s = 0
        m = []
        for p in range(P):
            v = int(b["match"][p, g])
            if v > la:
                s |= 2
                v = I64MIN
            m.append(v)
        if runs:
            r0, r1 = int(b["run_off"][g]), int(b["run_off"][g + 1])
            rr = [(pi if r == r0 else max(int(b["run_start"][r]), pi),
                   int(b["run_start"][r + 1]) - 1 if r + 1 < r1 else la, int(b["run_conf"][r]))
                  for r in range(r0, r1)]
        else:
            rr = [(pi, la, int(b["conf"][g]))]
        best = lc
        for (s0, e, cw) in rr:
            e = min(e, la)
            if e < s0:
                continue
            nm, om, nq, oq = cw & 0xFFFF, (cw >> 16) & 0xFFFF, (cw >> 32) & 0xFF, (cw >> 40) & 0xFF
            if nm == 0:
                s |= 4
            kn = I64MAX if nq == 0 else kth(m, nm, nq)
            ko = I64MAX if oq == 0 else kth(m, om, oq)
            cand = min(e, kn, ko)
            if cand >= s0:
                best = max(best, cand)
        out.append(best)
        st.append(s)
    return np.array(out, np.int64), np.array(st, np.uint8)


def replay(oracle, b, runs=True, chunk=7):
    kw = dict(run_off=b["run_off"], run_start=b["run_start"], run_conf=b["run_conf"]) if runs else {}
    c, s, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                         b["last_committed"], b["conf"], chunk=chunk, **kw)
    return c, s


def test_even_removal(oracle):
    b = even_removal_batch()
    c, s = replay(oracle, b)
    assert c[0] == 15
    mc, ms = model(b)
    assert mc[0] == 15 and ms[0] == s[0]


@pytest.mark.parametrize("P,seed", [(1, 1), (3, 2), (4, 3), (5, 4), (8, 5), (16, 6)])
def test_model_matches_replay(oracle, P, seed):
    b = random_batch(seed, 400, P)
    c, s = replay(oracle, b, chunk=int(seed % 5) + 1)
    mc, ms = model(b)
    np.testing.assert_array_equal(mc, c)
    np.testing.assert_array_equal(ms, s)


def test_ack_chunking_and_order_do_not_matter(oracle):
    """The reference's commit after an epoch is independent of how acks are chunked and
    interleaved (BallotBox.commitAt grants are idempotent; commit = max granted index)."""
    b = random_batch(42, 300, 5)
    base = replay(oracle, b, chunk=1)
    for ch in (2, 3, 64, 1024):
        np.testing.assert_array_equal(replay(oracle, b, chunk=ch)[0], base[0])


def scan_model(s):
    """The K-epoch kernel's formulation (quorum.hip quorum_epochs_kernel): per epoch an
    independent candidate v_k thresholded at pi_0, committed_k = max(lc_0, prefix max of v),
    pendingIndex before epoch k = committed_{k-1} + 1 once a commit happened."""
    K, P, G = s["match"].shape
    out = np.zeros((K, G), np.int64)
    st = np.zeros((K, G), np.uint8)
    for g in range(G):
        pi0, lc0 = int(s["pending_index"][g]), int(s["last_committed"][g])
        r0, r1 = int(s["run_off"][g]), int(s["run_off"][g + 1])
        runs = [(int(s["run_start"][r]), int(s["run_conf"][r])) for r in range(r0, r1)]
        M = I64MIN
        for k in range(K):
            la = int(s["last_appended"][k, g])
            if pi0 == 0:
                out[k, g], st[k, g] = lc0, 1
                continue
            pik = M + 1 if M > lc0 else pi0
            flags = 0
            m = []
            for p in range(P):
                v = int(s["match"][k, p, g])
                if v > la:
                    flags |= 2
                    v = I64MIN
                m.append(v)
            v = I64MIN
            for i, (start, cw) in enumerate(runs):
                thr = pi0 if i == 0 else max(start, pi0)
                end = runs[i + 1][0] - 1 if i + 1 < len(runs) else la
                ee = min(end, la)
                nm, om, nq, oq = cw & 0xFFFF, (cw >> 16) & 0xFFFF, (cw >> 32) & 0xFF, (cw >> 40) & 0xFF
                kn = I64MAX if nq == 0 else kth(m, nm, nq)
                ko = I64MAX if oq == 0 else kth(m, om, oq)
                cand = min(ee, kn, ko)
                if cand >= thr:
                    v = max(v, cand)
                sk = pik if i == 0 else max(start, pik)
                if ee >= sk and nm == 0:
                    flags |= 4
            M = max(M, v)
            out[k, g], st[k, g] = max(lc0, M), flags
    return out, st


@pytest.mark.parametrize("P,seed", [(3, 11), (5, 12), (2, 13)])
def test_epoch_scan_model_matches_sequential_replays(oracle, P, seed):
    """The thresholded prefix max over epochs equals K sequential BallotBox replays with the
    state carried between them (BallotBox.java:131-134), conf runs included."""
    from quorum_cases import random_series, series_replay
    s = random_series(seed, 300, P, 9)
    ce, se = series_replay(oracle, s)
    mc, ms = scan_model(s)
    np.testing.assert_array_equal(mc, ce)
    np.testing.assert_array_equal(ms, se)
    assert (ce[-1] > ce[0]).any()
