"""ctypes binding of libjrq.so (include/jrq.h).

This is the same C ABI a JDK 8 JNI shim binds; Python uses it
for tests and bench.py.  There is no CPU fallback: if libjrq.so is missing or no
gfx950 device is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JRQ_LIB") or os.path.join(os.path.dirname(_PKG), "lib", "libjrq.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_PKG)), "include", "jrq.h")

JRQ_OK = 0
ERRORS = {-1: "JRQ_E_INVALID", -2: "JRQ_E_NOMEM", -3: "JRQ_E_HIP", -4: "JRQ_E_RCCL",
          -5: "JRQ_E_NODEV", -6: "JRQ_E_STATE"}
ST_OK, ST_NOT_LEADER, ST_OUT_OF_RANGE, ST_EMPTY_CONF = 0, 1, 2, 4
FAN_NONE, FAN_APPLY, FAN_SKIP, FAN_INVALID = 0, 1, 2, 3  # jrq_fanout_status
V2_OK, V2_NULL, V2_V1, V2_HOST = 0, 1, 2, 3  # jrq_v2_status
MAX_PEERS = 16
CONF_RUNS = 1 << 63  # JRQ_CONF_RUNS: the group's pending window holds several conf runs


class JrqError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class GroupTiles(C.Structure):
    """jrq_group_tiles (include/jrq.h)."""
    _fields_ = [("tiles", C.c_void_p), ("num_peers", C.c_uint32), ("run_off", C.c_void_p),
                ("run_start", C.c_void_p), ("run_conf", C.c_void_p)]


class GroupBatch(C.Structure):
    """jrq_group_batch (include/jrq.h)."""
    _fields_ = [
        ("match", C.c_void_p),
        ("pending_index", C.c_void_p),
        ("last_appended", C.c_void_p),
        ("last_committed", C.c_void_p),
        ("conf", C.c_void_p),
        ("run_off", C.c_void_p),
        ("run_start", C.c_void_p),
        ("run_conf", C.c_void_p),
        ("num_peers", C.c_uint32),
        ("num_runs", C.c_uint32),
        ("match_ld", C.c_uint64),
    ]


TABLE_MAX_RUNS = 4                     # JRQ_TABLE_MAX_RUNS
TABLE_MAX_GROUPS = 1 << 27             # JRQ_TABLE_MAX_GROUPS
PI_FOLLOWS_LC = -(1 << 63)             # JRQ_PI_FOLLOWS_LC
REC_LAST_APPENDED = 16                 # JRQ_REC_LAST_APPENDED
TABLE_SLICE = 128                      # JRQ_TABLE_SLICE
STATE_RESET_MATCH = 1                  # JRQ_STATE_RESET_MATCH
STATE_STAMP = 2                        # JRQ_STATE_STAMP
READINDEX_PENDING, READINDEX_SUCCESS, READINDEX_FAILURE, READINDEX_INVALID = 0, 1, 2, 3  # JRQ_READINDEX_*
# jrq_debug_option (test / A-B hooks)
DBG_CRC_SEG_BYTES, DBG_CRC_REGS, DBG_CRC_PRIO, DBG_CRC_SEG_MAP, DBG_UPLOAD_PAGEABLE = 1, 2, 3, 4, 5

try:
    import numpy as _np
    # jrq_group_state (96 bytes)
    GROUP_STATE = _np.dtype([("group", "<u4"), ("num_runs", "<u2"), ("flags", "<u2"),
                             ("pending_index", "<i8"), ("last_appended", "<i8"),
                             ("last_committed", "<i8"), ("run_conf", "<u8", (TABLE_MAX_RUNS,)),
                             ("run_start", "<i8", (TABLE_MAX_RUNS,))])
    assert GROUP_STATE.itemsize == 96
except ImportError:  # pragma: no cover
    GROUP_STATE = None


class TableView(C.Structure):
    """jrq_table_view (include/jrq.h)."""
    _fields_ = [("match", C.c_void_p), ("pending_index", C.c_void_p),
                ("last_appended", C.c_void_p), ("last_committed", C.c_void_p),
                ("conf", C.c_void_p), ("ld", C.c_uint64), ("G", C.c_uint32),
                ("num_peers", C.c_uint32), ("tile_groups", C.c_uint32), ("tile_stride", C.c_uint64)]


def ack(group, field, index):
    """JRQ_ACK(group, field, index) -- vectorised: the low 32 bits of the absolute index."""
    import numpy as np
    g = np.asarray(group, dtype=np.uint64)
    f = np.asarray(field, dtype=np.uint64)
    lo = np.asarray(index, dtype=np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)
    return (lo << np.uint64(32)) | (g << np.uint64(5)) | f


def rec(group, field, v):
    """JRQ_REC(group, field, v) -- vectorised over numpy arrays."""
    import numpy as np
    g = np.asarray(group, dtype=np.uint64)
    f = np.asarray(field, dtype=np.uint64)
    vv = np.asarray(v, dtype=np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)
    return (vv << np.uint64(32)) | (g << np.uint64(5)) | f


# (name, restype, argtypes) for every function declared in include/jrq.h
_V = C.c_void_p
SIGNATURES = [
    ("jrq_abi_version", C.c_int, []),
    ("jrq_build_id", C.c_char_p, []),
    ("jrq_last_error", C.c_char_p, [_V]),
    ("jrq_create", _V, [C.c_int, C.c_uint32, C.c_uint8, C.POINTER(C.c_int)]),
    ("jrq_destroy", None, [_V]),
    ("jrq_get_stream", _V, [_V]),
    ("jrq_set_stream", C.c_int, [_V, _V]),
    ("jrq_synchronize", C.c_int, [_V]),
    ("jrq_host_register", C.c_int, [_V, C.c_size_t]),
    ("jrq_host_unregister", C.c_int, [_V]),
    ("jrq_host_alloc", C.c_int, [C.c_size_t, C.POINTER(C.c_void_p)]),
    ("jrq_host_free", C.c_int, [_V]),
    ("jrq_host_registered_bytes", C.c_int, [_V, C.POINTER(C.c_size_t)]),
    ("jrq_debug_set", C.c_int, [_V, C.c_int, C.c_int64]),
    ("jrq_quorum_epoch_dev", C.c_int, [_V, C.POINTER(GroupBatch), _V, _V, C.c_uint32]),
    ("jrq_quorum_epoch_tiles_dev", C.c_int, [_V, C.POINTER(GroupTiles), _V, _V, C.c_uint32]),
    ("jrq_quorum_epoch", C.c_int, [_V, C.POINTER(GroupBatch), _V, _V, C.c_uint32]),
    ("jrq_quorum_epoch_tiles", C.c_int, [_V, C.POINTER(GroupTiles), _V, _V, C.c_uint32]),
    ("jrq_quorum_epochs_dev", C.c_int,
     [_V, C.POINTER(GroupBatch), C.c_uint32, C.c_uint64, C.c_uint64, _V, _V, C.c_uint32]),
    ("jrq_quorum_epochs_tiles_dev", C.c_int,
     [_V, C.POINTER(GroupTiles), C.c_uint32, C.c_uint64, _V, _V, C.c_uint32]),
    ("jrq_crc64_batch_dev", C.c_int, [_V, _V, _V, C.c_uint32, _V]),
    ("jrq_crc64_batch", C.c_int, [_V, _V, _V, C.c_uint32, _V]),
    ("jrq_crc64_fixed_dev", C.c_int, [_V, _V, C.c_uint64, C.c_uint32, _V]),
    ("jrq_crc64_stream_update_dev", C.c_int, [_V, _V, _V, _V, C.c_uint32]),
    ("jrq_crc64_stream_update", C.c_int, [_V, _V, _V, _V, C.c_uint32]),
    ("jrq_logentry_checksum_batch_dev", C.c_int,
     [_V, _V, _V, _V, _V, _V, _V, C.c_uint32, _V, _V, _V, _V]),
    ("jrq_logentry_checksum_batch", C.c_int,
     [_V, _V, _V, _V, _V, _V, _V, C.c_uint32, _V, _V, _V, _V]),
    ("jrq_logentry_checksum_fixed_dev", C.c_int,
     [_V, _V, _V, _V, _V, _V, C.c_uint64, C.c_uint32, _V, _V, _V, _V]),
    ("jrq_append_entries_verify_dev", C.c_int,
     [_V, C.c_uint32, _V, _V, C.c_uint32, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    ("jrq_append_entries_verify", C.c_int,
     [_V, C.c_uint32, _V, _V, C.c_uint32, _V, _V, _V, _V, _V, _V, _V, _V, _V, _V]),
    ("jrq_lease_check_dev", C.c_int,
     [_V, _V, C.c_uint64, C.c_uint32, _V, _V, C.c_uint32, C.c_int64, C.c_int64, _V, _V, _V]),
    ("jrq_lease_check", C.c_int,
     [_V, _V, C.c_uint64, C.c_uint32, _V, _V, C.c_uint32, C.c_int64, C.c_int64, _V, _V, _V]),
    ("jrq_readindex_quorum_dev", C.c_int, [_V, _V, _V, _V, _V, C.c_uint32, C.c_uint32, _V]),
    ("jrq_readindex_quorum", C.c_int, [_V, _V, _V, _V, _V, C.c_uint32, C.c_uint32, _V]),
    ("jrq_leader_tick_dev", C.c_int,
     [_V, _V, C.c_uint64, C.c_uint32, _V, _V, C.c_uint32, C.c_int64, C.c_int64, _V, _V, _V, _V, _V, _V]),
    ("jrq_leader_tick", C.c_int,
     [_V, _V, C.c_uint64, C.c_uint32, _V, _V, C.c_uint32, C.c_int64, C.c_int64, _V, _V, _V, _V, _V, _V]),
    ("jrq_commit_fanout_dev", C.c_int, [_V, C.c_uint32] + [_V] * 9),
    ("jrq_commit_fanout", C.c_int, [_V, C.c_uint32] + [_V] * 9),
    ("jrq_v2_decode_verify_dev", C.c_int, [_V, _V, _V, C.c_uint32] + [_V] * 11),
    ("jrq_v2_decode_verify", C.c_int, [_V, _V, _V, C.c_uint32] + [_V] * 11),
    ("jrq_table_create", _V, [_V, C.c_uint32, C.c_uint32, C.POINTER(C.c_int)]),
    ("jrq_table_destroy", None, [_V]),
    ("jrq_table_update", C.c_int, [_V, _V, C.c_uint32, _V, C.c_uint32]),
    ("jrq_table_update_dev", C.c_int, [_V, _V, C.c_uint32, _V, C.c_uint32]),
    ("jrq_table_update_gather", C.c_int, [_V, C.c_uint32, _V, _V, _V, _V]),
    ("jrq_table_stage_reserve", C.c_int, [_V, C.c_uint32, C.c_uint32]),
    ("jrq_table_stage", C.c_int, [_V, _V, C.c_uint32, _V, C.c_uint32]),
    ("jrq_table_stage_apply", C.c_int, [_V]),
    ("jrq_table_epoch_dev", C.c_int, [_V, _V, _V, _V]),
    ("jrq_table_epoch", C.c_int, [_V, _V, _V, _V]),
    ("jrq_table_slices", C.c_uint32, [_V]),
    ("jrq_table_stage_reserve_acks", C.c_int, [_V, C.c_uint32, C.c_uint32]),
    ("jrq_table_committed_dev", C.c_int, [_V, _V]),
    ("jrq_table_ack_region", C.c_int, [_V, C.c_uint64, _V]),
    ("jrq_table_ack_region_free", C.c_int, [_V, _V]),
    ("jrq_table_ack_push", C.c_int, [_V, _V, _V, C.c_uint32]),
    ("jrq_table_stage_acks_dev", C.c_int, [_V, C.c_uint64, _V, C.c_uint32]),
    ("jrq_table_fsm_update", C.c_int, [_V, _V, _V, _V, _V, C.c_uint32]),
    ("jrq_table_fsm_update_dev", C.c_int, [_V, _V, _V, _V, _V, C.c_uint32]),
    ("jrq_table_fsm_read", C.c_int, [_V, _V, _V, _V]),
    ("jrq_table_epoch_fanout", C.c_int, [_V, _V, _V, _V, _V]),
    ("jrq_table_epoch_fanout_dev", C.c_int, [_V, _V, _V, _V, _V]),
    ("jrq_rccl_init_all", C.c_int, [_V, C.c_int]),
    ("jrq_publish_committed_all_dev", C.c_int, [_V, C.c_int, _V, _V, C.c_uint64]),
    ("jrq_snapshot_create", _V, [_V, C.c_int, C.POINTER(C.c_int)]),
    ("jrq_snapshot_destroy", None, [_V]),
    ("jrq_snapshot_publish", C.c_int, [_V]),
    ("jrq_snapshot_read", C.c_int, [_V, C.c_int, _V]),
    ("jrq_snapshot_via", C.c_int, [_V]),
    ("jrq_table_stage_acks", C.c_int, [_V, C.c_uint64, _V, C.c_uint32]),
    ("jrq_table_read", C.c_int, [_V, _V, _V, _V, _V]),
    ("jrq_table_check", C.c_int, [_V]),
    ("jrq_table_copy", C.c_int, [_V, _V]),
    ("jrq_table_view_get", C.c_int, [_V, C.POINTER(TableView)]),
    ("jrq_rccl_get_unique_id", C.c_int, [_V]),
    ("jrq_rccl_init", C.c_int, [_V, C.c_int, C.c_int, _V]),
    ("jrq_rccl_nranks", C.c_int, [_V]),
    ("jrq_publish_committed_dev", C.c_int, [_V, _V, _V, C.c_uint64]),
]

_lib = None


def load() -> C.CDLL:
    """Load libjrq.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7 /
        # libhsa-runtime64.so.1 / librccl.so.1 (same SONAMEs as /opt/rocm's).  Whichever
        # is loaded first is the one every later library binds to; if libjrq pulled in
        # /opt/rocm's first, torch would then find no GPU.  So load torch's first when
        # torch is installed (tensors, streams and libjrq then share one runtime).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        # (tools only: tools/gpu_check.sh's A/B runs point the bench at a variant build,
        # ab/<name>/libjrq.so; never set by the tests, smoke() or the driver's bench)
        path = os.environ.get("JRAFT_AMD_AB_LIB") or LIB_PATH
        if not os.path.exists(path):
            raise FileNotFoundError(
                f"{path} missing: run `make -C sofa-jraft_amd` (or __graft_entry__.build())")
        lib = C.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def build_id() -> str:
    """jrq_build_id() of the loaded library: the hash of the kernel sources it was built from."""
    return load().jrq_build_id().decode()


def check_build_id() -> str:
    """The loaded library's build id; raises unless it is the hash of the csrc/ beside it (the
    binary that runs is the one these sources make).  A/B variant libraries
    (JRAFT_AMD_AB_LIB) are built from edited copies and are exempt."""
    from ._srcsha import src_sha
    lib_sha, tree_sha = build_id(), src_sha()
    if lib_sha != tree_sha and not os.environ.get("JRAFT_AMD_AB_LIB"):
        raise RuntimeError(f"libjrq.so was built from other sources (jrq_build_id {lib_sha}, "
                           f"csrc/ hash {tree_sha}): rebuild with __graft_entry__.build()")
    return lib_sha


def check(rc: int, engine_handle=None) -> None:
    if rc != JRQ_OK:
        msg = load().jrq_last_error(engine_handle)
        raise JrqError(rc, msg.decode() if msg else "")


PAGE = 4096
_STILL_REGISTERED = []


def page_aligned_copy(a):
    """A copy of numpy array `a` that starts on a page and owns every page it touches (a
    DirectByteBuffer carved from an aligned slab): jrq_host_register never refuses it for a
    page shared with another registration, and freeing it frees no neighbour's page."""
    import numpy as np
    a = np.ascontiguousarray(a)
    n = a.nbytes
    buf = np.empty(((n + PAGE - 1) // PAGE) * PAGE + PAGE, np.uint8)
    off = (-buf.ctypes.data) % PAGE
    v = buf[off:off + n].view(a.dtype).reshape(a.shape)
    v[...] = a
    return v


def host_registrations():
    """(live ranges, their total bytes) in libjrq's page-lock registry."""
    n = C.c_size_t()
    k = load().jrq_host_registered_bytes(None, C.byref(n))
    return int(k), int(n.value)


class Registered:
    """Context manager: jrq_host_register every array (page-aligned copies from
    page_aligned_copy), unregister on exit and raise if any unregistration fails -- a
    registration left over freed memory is a stale device mapping of that address."""

    def __init__(self, arrays):
        self.arrays = list(arrays)
        self.live = []

    def __enter__(self):
        L = load()
        for a in self.arrays:
            rc = L.jrq_host_register(C.c_void_p(a.ctypes.data), a.nbytes)
            if rc != JRQ_OK:
                self.__exit__(None, None, None)
                raise JrqError(rc, f"jrq_host_register({a.nbytes} B at {a.ctypes.data:#x})")
            self.live.append(a)
        return self

    def __exit__(self, *exc):
        L = load()
        bad = []
        while self.live:
            a = self.live.pop()
            rc = L.jrq_host_unregister(C.c_void_p(a.ctypes.data))
            if rc != JRQ_OK:
                bad.append((a.ctypes.data, a.nbytes, ERRORS.get(rc, rc)))
                _STILL_REGISTERED.append(a)  # never freed while HIP may still map it
        if bad and exc[0] is None:
            raise JrqError(-3, f"jrq_host_unregister failed: {bad}")
        return False


def conf_word(new_mask: int, old_mask: int = 0, new_q: int | None = None,
              old_q: int | None = None, old_present: bool | None = None) -> int:
    """JRQ_CONF(): quorums default to Ballot.init's |conf|/2+1 (Ballot.java:77-83)."""
    if new_q is None:
        new_q = bin(new_mask).count("1") // 2 + 1
    if old_present is None:
        old_present = old_mask != 0 or (old_q is not None and old_q > 0)
    if old_q is None:
        old_q = (bin(old_mask).count("1") // 2 + 1) if old_present else 0
    return (new_mask & 0xFFFF) | ((old_mask & 0xFFFF) << 16) | ((new_q & 0xFF) << 32) | \
        ((old_q & 0xFF) << 40)
