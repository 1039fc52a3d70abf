"""GPU: host-variant uploads of caller memory (the DirectByteBuffer path of INTEGRATION.md).

Round 2 saw two "illegal memory access" errors reported by a host variant's upload of a
read-only > 1 MiB numpy view over a Python bytes object, after a successful stream
synchronisation; the uploads were then routed through the engine's pinned bounce chunks.
These tests pin the cases down, each followed by conftest's device-wide synchronisation:
  * the default path (bounce chunks) on read-only views of 1 MiB + 1 .. 64 MiB,
  * HIP's own pageable copy on the same views (JRQ_DBG_UPLOAD_PAGEABLE), the path that failed,
  * caller memory registered with jrq_host_register (DMA straight from the caller's pages).
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
