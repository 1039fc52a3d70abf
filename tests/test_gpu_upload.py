"""GPU: host-variant uploads of caller memory (the DirectByteBuffer path of INTEGRATION.md).

Rounds 2 and 3 saw "illegal memory access" errors reported by a > 1 MiB pageable upload (a host
variant's, then torch's) after a successful device synchronisation.  Round 3 traced the trigger
to hipHostRegister / hipHostUnregister called from several threads at once (the host mirror's
pack workers registering their staging buffers): the failing drive test passed once the same
buffers were registered from one thread.  libjrq now serialises its pin calls.
These tests pin the cases down, each followed by conftest's device-wide synchronisation:
  * the default path (bounce chunks) on read-only views of 1 MiB + 1 .. 64 MiB,
  * HIP's own pageable copy on the same views (JRQ_DBG_UPLOAD_PAGEABLE),
  * caller memory registered with jrq_host_register (DMA straight from the caller's pages),
  * registrations from 16 threads at once, then pageable uploads of fresh arrays.
"""
import numpy as np
import pytest

from jraft_amd import _lib
from jraft_amd import workloads as W
from devio import host_np, to_dev

pytestmark = pytest.mark.gpu

SIZES = [(1 << 20) + 1, 4 << 20, (16 << 20) + 13, 64 << 20]


def _readonly_view(seed, n):
    v = np.frombuffer(W.random_bytes(seed, n).tobytes(), np.uint8)  # over a bytes object
    assert not v.flags.writeable
    return v


def _entries(n):
    """DATA entries of ragged sizes covering n bytes (the last one takes the rest)."""
    offs = W.ragged_offsets(n, max(1, n // 9000), 16000)
    offs = offs[offs < n]
    return np.append(offs, n).astype(np.uint64)


@pytest.mark.parametrize("pageable", [0, 1], ids=["bounce", "hip_pageable"])
@pytest.mark.parametrize("n", SIZES)
def test_readonly_view_uploads(oracle, n, pageable):
    from jraft_amd import Engine
    payload = _readonly_view(n, n)
    offs = _entries(n)
    m = len(offs) - 1
    et = np.full(m, 2, np.uint8)
    idx = np.arange(1, m + 1, dtype=np.int64)
    term = np.ones(m, np.int64)
    exp = oracle.logentry_checksum_batch(et, idx, term, None, payload, offs)
    with Engine(0) as e:
        e.debug_set(_lib.DBG_UPLOAD_PAGEABLE, pageable)
        for _ in range(2):
            np.testing.assert_array_equal(e.logentry_checksum_batch(et, idx, term, None, payload, offs), exp)
            np.testing.assert_array_equal(e.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))
            e.synchronize()


def test_registered_caller_buffer(oracle):
    """A jrq_host_register'ed caller buffer (a pinned DirectByteBuffer) is DMA-ed directly."""
    import ctypes

    from jraft_amd import Engine
    n = 24 << 20
    buf = np.empty(n + 4096, np.uint8)
    a = buf[(-buf.ctypes.data) % 4096:][:n]   # page-aligned, as a DirectByteBuffer
    a[:] = W.random_bytes(3, n)
    L = _lib.load()
    assert L.jrq_host_register(ctypes.c_void_p(a.ctypes.data), n) == 0
    try:
        offs = np.arange(0, n + 1, 16384, dtype=np.uint64)
        with Engine(0) as e:
            np.testing.assert_array_equal(e.crc64_batch(a, offs), oracle.crc64_batch(a, offs))
    finally:
        assert L.jrq_host_unregister(ctypes.c_void_p(a.ctypes.data)) == 0


def test_concurrent_registrations_then_pageable_uploads(oracle):
    """16 threads register, use and unregister their own buffers through jrq_host_register at
    the same time (as the mirror's pack workers once did, and as a JNI host pinning
    DirectByteBuffers from its RPC threads may); afterwards fresh > 1 MiB arrays go up through
    torch's pageable copy and through the host variants, and come back intact."""
    import ctypes
    import threading

    import torch

    from jraft_amd import Engine
    L = _lib.load()
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(t)
            for _ in range(4):
                n = int(rng.integers(1, 9)) << 20
                buf = np.empty(n + 4096, np.uint8)
                a = buf[(-buf.ctypes.data) % 4096:][:n]
                a[:] = t
                if L.jrq_host_register(ctypes.c_void_p(a.ctypes.data), n) != 0:
                    errors.append(("register", t, n))
                    continue
                if L.jrq_host_unregister(ctypes.c_void_p(a.ctypes.data)) != 0:
                    errors.append(("unregister", t, n))
                del a, buf
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(repr(ex))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    dev = torch.device("cuda:0")
    # after the registration churn HIP must hold no registration over fresh memory (a stale
    # one is what the rounds 2-3 fault DMA-ed through); round trips through page-locked memory
    from conftest import assert_unregistered
    for k in range(6):
        host = np.frombuffer(W.random_bytes(100 + k, (8 << 20) + 8 * k), np.int64).copy()
        assert_unregistered({"host": host}, "after concurrent register/unregister")
        got = host_np(to_dev(host, dev))
        np.testing.assert_array_equal(got, host)
    payload = W.random_bytes(7, 6 << 20)
    offs = np.arange(0, len(payload) + 1, 4096, dtype=np.uint64)
    with Engine(0) as e:
        np.testing.assert_array_equal(e.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))


def test_registry_refuses_shared_pages_and_unknown_ranges(oracle):
    """libjrq tracks registrations by page: a range sharing a page with a live one is refused
    (JRQ_E_STATE, nothing pinned), so no page is mapped twice; unregistering a pointer that is
    not the start of a live jrq_host_register range is refused (JRQ_E_INVALID) without calling
    HIP; a refused buffer still uploads correctly, through the bounce chunks."""
    import ctypes

    from jraft_amd import Engine
    L = _lib.load()
    base = _lib.host_registrations()
    buf = np.empty(6 * 4096, np.uint8)
    a0 = (-buf.ctypes.data) % 4096
    first = buf[a0:a0 + 4096 + 100]                  # pages 0 and 1
    second = buf[a0 + 4096 + 200:a0 + 3 * 4096]       # pages 1 and 2: shares page 1
    third = buf[a0 + 2 * 4096:a0 + 4 * 4096]         # pages 2 and 3: free of `first`
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)    # noqa: E731
    assert L.jrq_host_register(vp(first), first.nbytes) == 0
    try:
        assert L.jrq_host_register(vp(second), second.nbytes) == -6   # JRQ_E_STATE
        assert _lib.host_registrations() == (base[0] + 1, base[1] + first.nbytes)
        assert L.jrq_host_unregister(vp(second)) == -1                # never registered
        assert L.jrq_host_unregister(ctypes.c_void_p(first.ctypes.data + 8)) == -1  # interior
        assert L.jrq_host_free(vp(first)) == -1                       # not a jrq_host_alloc block
        assert L.jrq_host_register(vp(third), third.nbytes) == 0
        assert L.jrq_host_unregister(vp(third)) == 0
        # the refused range's upload takes the bounce chunks and is still right
        second[:] = W.random_bytes(11, second.nbytes)
        offs = np.array([0, 777, second.nbytes], np.uint64)
        with Engine(0) as e:
            np.testing.assert_array_equal(e.crc64_batch(second, offs), oracle.crc64_batch(second, offs))
    finally:
        assert L.jrq_host_unregister(vp(first)) == 0
    assert L.jrq_host_unregister(vp(first)) == -1                     # already gone
    assert _lib.host_registrations() == base
    p = ctypes.c_void_p()
    assert L.jrq_host_alloc(10000, ctypes.byref(p)) == 0
    assert _lib.host_registrations()[0] == base[0] + 1
    assert L.jrq_host_unregister(p) == -1                             # alloc'ed, not registered
    assert L.jrq_host_free(p) == 0
    assert _lib.host_registrations() == base


def test_pinned_then_c1_then_lease_legs(engine):
    """The bench sequence of round 4's one unexplained fault: the pinned leg
    (every C5 / C1 input registered, used, unregistered), then C1, then the lease leg, whose
    result copies faulted once.  The registry must be back at its size before the pinned leg,
    HIP must know no registration over fresh arrays of the lease results' sizes, and both later
    legs must be bit-exact against the oracle."""
    import os
    import sys
    import types

    import torch

    from conftest import assert_unregistered, device_checkpoint
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, ROOT)
    import bench
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    args = types.SimpleNamespace(steps=5, warmup=1, no_cpu=False)
    base = _lib.host_registrations()
    old = bench.WARM_MS
    bench.WARM_MS = 5.0
    try:
        with torch.cuda.stream(stream):
            engine.use_stream(stream.cuda_stream)
            ctx = bench.Ctx(engine, stream, dev, 1, 0, args)
            _, _, c5state = bench.leg_c5(ctx, args, lambda: None, lambda x: x, time_it=False)
            pin = bench.leg_pinned(ctx, args, c5state)
            del c5state
            for name in ("C5", "C1"):
                for how in ("registered", "unregistered"):
                    assert pin[name][how]["bit_exact_vs_oracle"] is True, (name, how)
            assert pin["C5"]["registered"]["registered_arrays"] == 6
            assert _lib.host_registrations() == base
            device_checkpoint("after the pinned leg")
            c1 = bench.leg_c1(ctx, args)
            assert c1["bit_exact_vs_oracle"] is True
            G = 1 << 20
            fresh = {"ok": np.empty(G, np.uint8), "lead": np.empty(G, np.int64),
                     "dead": np.empty(G, np.int16), "ts": np.empty((5, G), np.int64)}
            assert_unregistered(fresh, "before the lease leg")
            del fresh
            from jraft_amd import workloads as W
            conf = W.quorum_batch("C3", groups=G)["conf"]
            lease = bench.leg_lease(ctx, args, bench.to_dev(conf, dev), G, 5)
            assert lease["bit_exact_vs_oracle"] is True
            torch.cuda.synchronize()
    finally:
        bench.WARM_MS = old
        engine.use_stream(None)
    assert _lib.host_registrations() == base


def test_result_downloads_through_bounce_chunks(engine):
    """Host-variant results land in caller memory that is not page-locked through the engine's
    8 MiB bounce chunks (several chunks here: 1.5M groups = 12 MB of commits), never through a
    HIP pageable copy; they equal the device entry point's results, copied out through
    page-locked memory."""
    import torch
    b = W.quorum_batch("C2", groups=1_500_000)
    c_host, s_host = engine.quorum_epoch(b["match"], b["pending_index"], b["last_appended"],
                                         b["last_committed"], b["conf"])
    dev = torch.device("cuda:0")
    t = {k: to_dev(v, dev) for k, v in b.items()}
    G = b["pending_index"].shape[0]
    out = torch.empty(G, dtype=torch.int64, device=dev)
    st = torch.empty(G, dtype=torch.uint8, device=dev)
    engine.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"], t["last_committed"],
                            t["conf"], out, st)
    engine.synchronize()
    h = torch.empty(G, dtype=torch.int64, pin_memory=True)
    h.copy_(out)
    hs = torch.empty(G, dtype=torch.uint8, pin_memory=True)
    hs.copy_(st)
    assert np.array_equal(c_host, h.numpy()) and np.array_equal(s_host, hs.numpy())
    assert (c_host >= b["last_committed"]).all()
