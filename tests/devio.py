"""Device <-> host transfers for the GPU tests, always through page-locked host memory.

No HIP copy in the tests, smoke or bench takes pageable memory: HIP copies a
large pageable range by locking the caller's pages itself and keeps that lock, found again by
address, after the copy returns; memory freed and allocated again at the same address is then
DMA-ed through a lock over pages that are gone -- the "illegal memory access" of rounds 2-5.
These are the tests' equivalents of bench.to_dev / bench.host_np.
"""
import numpy as np


def to_dev(a, dev="cuda:0"):
    """A device tensor holding numpy array `a` (uint64 as int64 words, uint16 as int16),
    uploaded from a page-locked copy."""
    import torch
    if a is None:
        return None
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint16:
        a = a.view(np.int16)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    if not a.flags.writeable:
        a = a.copy()
    return torch.from_numpy(a).pin_memory().to(dev)


def host_t(t):
    """A page-locked host copy of device tensor `t` (same shape and dtype)."""
    import torch
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h


def host_np(t):
    """numpy copy of device tensor `t`, downloaded into page-locked memory."""
    return host_t(t).numpy()
