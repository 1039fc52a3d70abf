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
    for k in range(6):
        host = np.frombuffer(W.random_bytes(100 + k, (8 << 20) + 8 * k), np.int64).copy()
        got = torch.from_numpy(host).to(dev).cpu().numpy()
        np.testing.assert_array_equal(got, host)
    payload = W.random_bytes(7, 6 << 20)
    offs = np.arange(0, len(payload) + 1, 4096, dtype=np.uint64)
    with Engine(0) as e:
        np.testing.assert_array_equal(e.crc64_batch(payload, offs), oracle.crc64_batch(payload, offs))
