import ctypes
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sofa-jraft_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libjrq.so")


@pytest.fixture(scope="session")
def oracle():
    import jraft_oracle
    jraft_oracle.lib()
    return jraft_oracle


@pytest.fixture(scope="session")
def engine():
    """One libjrq engine on cuda:0 for the whole GPU session (fails loudly without one)."""
    from jraft_amd import Engine
    e = Engine(0)
    yield e
    e.close()


_hip = None


def _hip_runtime():
    """The HIP runtime libjrq and torch share in this process (loaded by jraft_amd._lib)."""
    global _hip
    if _hip is None:
        from jraft_amd import _lib
        _lib.load()
        # already loaded (torch's copy, SONAME libamdhip64.so.7): NOLOAD binds that one
        _hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
        _hip.hipDeviceSynchronize.restype = ctypes.c_int
        _hip.hipGetLastError.restype = ctypes.c_int
        _hip.hipGetErrorString.restype = ctypes.c_char_p
        _hip.hipGetErrorString.argtypes = [ctypes.c_int]
    return _hip


class _PtrAttr(ctypes.Structure):  # hipPointerAttribute_t (hip_runtime_api.h)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int),
                ("devicePointer", ctypes.c_void_p), ("hostPointer", ctypes.c_void_p),
                ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def hip_registration(addr):
    """What HIP knows about host address `addr`: None for plain pageable memory, else the
    registration it finds there (type, device pointer, and the device range it belongs to)."""
    hip = _hip_runtime()
    a = _PtrAttr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(addr))
    hip.hipGetLastError()
    if rc or a.type == 0:
        return None
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    rr = hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size),
                                   ctypes.c_void_p(a.devicePointer))
    hip.hipGetLastError()
    return {"addr": hex(addr), "type": a.type, "devicePointer": hex(a.devicePointer or 0),
            "hostPointer": hex(a.hostPointer or 0), "flags": a.allocationFlags,
            "dev_range": None if rr else (hex(base.value or 0), size.value)}


def assert_unregistered(arrays, where):
    """Fail (before any copy) if HIP holds a registration over memory we never registered:
    a pageable copy from such an address would DMA through that stale mapping."""
    stale = []
    for name, a in arrays.items():
        if not hasattr(a, "ctypes") or a.nbytes == 0:
            continue
        for off in sorted({0, a.nbytes // 2, a.nbytes - 1}):
            r = hip_registration(a.ctypes.data + off)
            if r is not None:
                stale.append((name, a.nbytes, off, r))
    if stale:
        pytest.fail("HIP reports registrations over unregistered numpy arrays %s: %r"
                    % (where, stale), pytrace=False)


def device_checkpoint(where):
    """Synchronise the device now and fail naming `where` if it reports an error: inside a test
    with several GPU steps, it charges an asynchronous fault to the step that caused it."""
    hip = _hip_runtime()
    rc = hip.hipDeviceSynchronize()
    hip.hipGetLastError()
    if rc:
        pytest.fail("device error at %s: %s (hipDeviceSynchronize -> %d)"
                    % (where, hip.hipGetErrorString(rc).decode(), rc), pytrace=False)


@pytest.fixture(autouse=True)
def _device_fault_check(request):
    """After every GPU test: synchronise the whole device and check for an error.  A kernel
    fault is asynchronous -- on its own it surfaces at the next HIP call, possibly in another
    test (round 2 saw an "illegal memory access" reported by a later copy).  Synchronising
    here charges it to the test whose kernels caused it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    hip = _hip_runtime()
    rc = hip.hipDeviceSynchronize()
    # (hipGetLastError alone also holds expected API refusals, e.g. the engine's probe of an
    # unregistered pointer; only a failing device-wide synchronisation is a fault)
    hip.hipGetLastError()
    if rc:
        pytest.fail("device error after %s: %s (hipDeviceSynchronize -> %d)"
                    % (request.node.nodeid, hip.hipGetErrorString(rc).decode(), rc),
                    pytrace=False)
