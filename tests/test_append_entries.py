"""Follower verify on receive: the oracle's restatement of
NodeImpl.handleAppendEntriesRequest (NodeImpl.java:1766-1792) on CPU, and the GPU batch
(jrq_append_entries_verify) against it."""
import numpy as np
import pytest

from ae_cases import random_requests
from devio import to_dev, host_np


def test_oracle_follows_reference_loop(oracle):
    """index = prevLogIndex + 1 + i; UNKNOWN entries take no bytes; first corrupt wins."""
    payload = b"hello" + b"world!" + b"xyz"
    # request 0: NO_OP "hello", UNKNOWN (data_len 4 but consumes nothing), DATA "world!"
    # request 1: DATA "xyz"
    req_off = [0, 3, 4]
    prev = [99, 7]
    term = [3, 3, 3, 5]
    etype = [1, 0, 2, 2]
    data_len = [5, 4, 6, 3]
    exp = [oracle.logentry_checksum(1, 100, 3, 0, b"hello"),
           oracle.logentry_checksum(0, 101, 3, 0, b""),
           oracle.logentry_checksum(2, 102, 3, 0, b"world!"),
           oracle.logentry_checksum(2, 8, 5, 0, b"xyz")]
    data = np.frombuffer(payload, np.uint8)
    out, cor, first = oracle.append_entries_verify(req_off, prev, term, etype, data_len,
                                                   np.array(exp, np.uint64), data)
    assert [int(x) for x in out] == exp
    assert not cor.any() and list(first) == [-1, -1]
    bad = np.array(exp, np.uint64)
    bad[2] ^= np.uint64(5)
    bad[3] ^= np.uint64(1)
    _, cor, first = oracle.append_entries_verify(req_off, prev, term, etype, data_len, bad, data)
    assert list(cor) == [0, 0, 1, 1] and list(first) == [2, 0]
    # no checksum on the entry -> never corrupt (hasChecksum false)
    _, cor, first = oracle.append_entries_verify(req_off, prev, term, etype, data_len, bad, data,
                                                 has_checksum=[1, 1, 0, 1])
    assert list(first) == [-1, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("R,max_entries,max_len", [(1, 1, 10), (7, 64, 3000), (300, 100, 2000),
                                                   (50, 1024, 256), (3, 5, 200000)])
def test_gpu_matches_oracle(engine, oracle, R, max_entries, max_len):
    b = random_requests(R * 7 + max_len, R, max_entries, max_len, oracle=oracle)
    args = (b["req_off"], b["prev_log_index"], b["term"], b["etype"], b["data_len"],
            b["checksum"], b["data"])
    kw = dict(has_checksum=b["has_checksum"], peer_xor=b["peer_xor"])
    e_out, e_cor, e_first = oracle.append_entries_verify(*args, **kw)
    g_out, g_cor, g_first = engine.append_entries_verify(*args, **kw)
    np.testing.assert_array_equal(g_out, e_out)
    np.testing.assert_array_equal(g_cor, e_cor)
    np.testing.assert_array_equal(g_first, e_first)


@pytest.mark.gpu
def test_gpu_empty_requests(engine, oracle):
    req_off = np.array([0, 0, 0], np.uint32)
    out, cor, first = engine.append_entries_verify(req_off, [5, 6], [], [], [], [], None)
    assert list(first) == [-1, -1] and out.size == 0


@pytest.mark.gpu
@pytest.mark.parametrize("R,per,L,spoil", [(16, 256, 16384, None), (200, 1024, 256, None),
                                          (16, 256, 16384, "length"), (16, 256, 16384, "unknown"),
                                          (16, 256, 16384, "misaligned")])
def test_gpu_uniform_entries(engine, oracle, R, per, L, spoil):
    """Batches of one entry length, none UNKNOWN (a client's fixed-size commands: 16 KiB and
    256-B entries), and the same batches spoiled: one entry one byte shorter, one entry UNKNOWN,
    or (device entry point) a payload 8 bytes past a 16-B boundary.  All against the oracle,
    corrupt flags included.  (A fixed-size data path for such batches was measured and dropped
    in r05: its gate and the early-returning walk launches cost what the fixed kernel saved.)"""
    import torch
    b = random_requests(R + L, R, per, L, oracle=oracle, uniform=L)
    if spoil in ("length", "unknown"):
        i = len(b["data_len"]) // 3
        if spoil == "length":
            b["data_len"][i] -= 1
            b["data"] = np.delete(b["data"], int(b["data_len"][:i].sum()))
        else:
            b["etype"][i] = 0
            b["data"] = np.delete(b["data"], np.arange(int(b["data_len"][:i].sum()),
                                                       int(b["data_len"][:i + 1].sum())))
        good, _, _ = oracle.append_entries_verify(b["req_off"], b["prev_log_index"], b["term"],
                                                  b["etype"], b["data_len"], b["checksum"],
                                                  b["data"], has_checksum=np.zeros(len(b["term"]), np.uint8),
                                                  peer_xor=b["peer_xor"])
        b["checksum"] = good
        b["checksum"][::97] ^= np.uint64(1)
    args = (b["req_off"], b["prev_log_index"], b["term"], b["etype"], b["data_len"],
            b["checksum"], b["data"])
    kw = dict(has_checksum=b["has_checksum"], peer_xor=b["peer_xor"])
    e_out, e_cor, e_first = oracle.append_entries_verify(*args, **kw)
    assert e_cor.any()
    if spoil != "misaligned":
        g_out, g_cor, g_first = engine.append_entries_verify(*args, **kw)
    else:  # the device entry point on a payload 8 bytes past a 16-B boundary
        dev = torch.device("cuda:0")
        t = lambda a: to_dev(np.ascontiguousarray(a.view(np.int64) if a.dtype == np.uint64 else a), dev)
        buf = torch.zeros(b["data"].size + 16, dtype=torch.uint8, device=dev)
        buf[8:8 + b["data"].size] = to_dev(b["data"], dev)
        N, Rr = len(b["term"]), len(b["prev_log_index"])
        out = torch.empty(N, dtype=torch.int64, device=dev)
        cor = torch.empty(N, dtype=torch.uint8, device=dev)
        first = torch.empty(Rr, dtype=torch.int32, device=dev)
        engine.append_entries_verify_dev(t(b["req_off"].view(np.int32)), t(b["prev_log_index"]), t(b["term"]),
                                         t(b["etype"]), t(b["data_len"]), t(b["checksum"]), buf[8:],
                                         out, cor, first, has_checksum=t(b["has_checksum"]),
                                         peer_xor=t(b["peer_xor"]))
        engine.synchronize()
        g_out, g_cor, g_first = host_np(out).view(np.uint64), host_np(cor), host_np(first)
    np.testing.assert_array_equal(g_out, e_out)
    np.testing.assert_array_equal(g_cor, e_cor)
    np.testing.assert_array_equal(g_first, e_first)
