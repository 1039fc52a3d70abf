"""Python face of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker or the timed CPU baseline.  The
product path (``libjrq.so`` + ``jraft_amd``) never imports it.

Two layers:
  * ctypes bindings to ``oracle/_build/libjraft_oracle.so`` (jraft_oracle.c), the
    Java-faithful restatement used for parity and as the "port" CPU baseline;
  * tiny pure-Python restatements (``py_crc64`` ...) used only on small inputs to
    cross-check the C restatement itself.
Reference citations use JC = jraft-core/src/main/java/com/alipay/sofa/jraft.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libjraft_oracle.so")
_lib = None

POLY = 0x42F0E1EBA9EA3693  # JC/util/CRC64.java:27-40
M64 = (1 << 64) - 1

# status codes (shared with include/jrq.h)
ST_OK, ST_NOT_LEADER, ST_OUT_OF_RANGE, ST_EMPTY_CONF = 0, 1, 2, 4
FALSE, TRUE, AIOOBE, IAE = 0, 1, -1, -2

_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile the C oracle with make (gcc only)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.jo_crc64.restype = C.c_uint64
        L.jo_crc64.argtypes = [C.c_void_p, C.c_size_t]
        L.jo_crc64_update.restype = C.c_uint64
        L.jo_crc64_update.argtypes = [C.c_uint64, C.c_void_p, C.c_size_t]
        L.jo_crc64_table.restype = C.POINTER(C.c_uint64)
        L.jo_crc64_batch.restype = None
        L.jo_crc64_batch.argtypes = [_u8p, _u64p, C.c_uint32, _u64p]
        L.jo_logid_checksum.restype = C.c_uint64
        L.jo_logid_checksum.argtypes = [C.c_int64, C.c_int64]
        L.jo_peerid_checksum.restype = C.c_uint64
        L.jo_peerid_checksum.argtypes = [C.c_char_p, C.c_int32, C.c_int32]
        L.jo_logentry_checksum.restype = C.c_uint64
        L.jo_logentry_checksum.argtypes = [C.c_int32, C.c_int64, C.c_int64, C.c_uint64, C.c_void_p,
                                           C.c_size_t]
        L.jo_logentry_checksum_batch.restype = None
        L.jo_logentry_checksum_batch.argtypes = [_u8p, _i64p, _i64p, C.c_void_p, _u8p, _u64p,
                                                 C.c_uint32, _u64p, C.c_void_p, C.c_void_p,
                                                 C.c_void_p]
        L.jo_append_entries_verify.restype = None
        L.jo_append_entries_verify.argtypes = [C.c_uint32] + [C.c_void_p] * 12
        L.jo_lease_check.restype = None
        L.jo_lease_check.argtypes = [C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.jo_readindex_round.restype = C.c_uint8
        L.jo_readindex_round.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32]
        L.jo_readindex_quorum.restype = None
        L.jo_readindex_quorum.argtypes = [C.c_uint32, C.c_uint32] + [C.c_void_p] * 5
        L.jo_bb_new.restype = C.c_void_p
        L.jo_bb_free.argtypes = [C.c_void_p]
        for name in ("jo_bb_last_committed_index", "jo_bb_pending_index", "jo_bb_queue_size",
                     "jo_bb_on_committed_calls", "jo_bb_on_committed_last"):
            getattr(L, name).restype = C.c_int64
            getattr(L, name).argtypes = [C.c_void_p]
        L.jo_bb_commit_at.restype = C.c_int
        L.jo_bb_commit_at.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int32]
        L.jo_bb_clear_pending_tasks.argtypes = [C.c_void_p]
        L.jo_bb_reset_pending_index.restype = C.c_int
        L.jo_bb_reset_pending_index.argtypes = [C.c_void_p, C.c_int64]
        L.jo_bb_append_pending_task.restype = C.c_int
        L.jo_bb_append_pending_task.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p,
                                                C.c_int32]
        L.jo_bb_set_last_committed_index.restype = C.c_int
        L.jo_bb_set_last_committed_index.argtypes = [C.c_void_p, C.c_int64]
        L.jo_quorum_epoch_replay.restype = C.c_int64
        L.jo_quorum_epoch_replay.argtypes = [C.c_uint32, C.c_uint32, _i64p, _i64p, _i64p, _i64p,
                                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_int64, _i64p, _u8p]
        L.jo_v2_decode_batch.restype = None
        L.jo_v2_decode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32] + [C.c_void_p] * 11
        L.jo_v2_peer_checksum.restype = C.c_uint64
        L.jo_v2_peer_checksum.argtypes = [C.c_char_p, C.c_int64, C.POINTER(C.c_int)]
        L.jo_commit_fanout_replay.restype = C.c_int64
        L.jo_commit_fanout_replay.argtypes = [C.c_uint32] + [C.c_void_p] * 7
        # cpu_fast.c: optimised CPU baselines (bench.py), checked against the above
        L.jo_fast_crc64_batch.restype = None
        L.jo_fast_crc64_batch.argtypes = [_u8p, _u64p, C.c_uint32, _u64p]
        L.jo_fast_quorum_epoch.restype = None
        L.jo_fast_quorum_epoch.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64] + [C.c_void_p] * 7
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ------------------------------------------------------------------ CRC64 --

def table() -> np.ndarray:
    t = lib().jo_crc64_table()
    return np.array([t[i] for i in range(256)], dtype=np.uint64)


def crc64(data: bytes) -> int:
    """CrcUtil.crc64(byte[]) (JC/util/CrcUtil.java:36-41); None -> 0 as in the reference."""
    if data is None:
        return 0
    b = bytes(data)
    return int(lib().jo_crc64(C.c_char_p(b), len(b)))


def crc64_batch(payload: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.zeros(max(n, 0), dtype=np.uint64)
    if n > 0:
        if payload.size == 0:
            payload = np.zeros(1, dtype=np.uint8)
        lib().jo_crc64_batch(payload, offsets, n, out)
    return out


def crc64_stream_update(state: np.ndarray, payload: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """S streaming java.util.zip.Checksum objects (`new CRC64()`, JC/util/CRC64.java:26), each
    fed one chunk by CRC64.update(byte[],off,len) (:106-110) starting from register state[s],
    as CheckedOutputStream/CheckedInputStream do around ZipUtil.compress/decompress
    (RK/util/ZipUtil.java:45-94; RK/storage/AbstractKVStoreSnapshotFile.java:121,139).
    Returns the registers after the chunks (getValue(), :119-121)."""
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    out = np.array(state, dtype=np.uint64, copy=True)
    L = lib()
    base = payload.ctypes.data
    for s in range(len(offsets) - 1):
        o0, o1 = int(offsets[s]), int(offsets[s + 1])
        out[s] = L.jo_crc64_update(int(out[s]), C.c_void_p(base + o0), o1 - o0)
    return out


def fast_crc64_batch(payload: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """Slice-by-8 CRC64 (cpu_fast.c): the optimised-CPU baseline, same results as crc64_batch."""
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    out = np.zeros(max(n, 0), dtype=np.uint64)
    if n > 0:
        lib().jo_fast_crc64_batch(payload if payload.size else np.zeros(1, np.uint8), offsets, n, out)
    return out


def fast_quorum_epoch(match, pending_index, last_appended, last_committed, conf):
    """Closed-form epoch per group (cpu_fast.c): the optimised-CPU quorum baseline."""
    match = np.ascontiguousarray(match, dtype=np.int64)
    P, G = match.shape
    arrs = [np.ascontiguousarray(a, dtype=np.int64) for a in (pending_index, last_appended,
                                                               last_committed)]
    conf = np.ascontiguousarray(conf, dtype=np.uint64)
    committed = np.empty(G, np.int64)
    status = np.empty(G, np.uint8)
    lib().jo_fast_quorum_epoch(P, G, G, _ptr(match), *[_ptr(a) for a in arrs], _ptr(conf),
                               _ptr(committed), _ptr(status))
    return committed, status


def logid_checksum(index: int, term: int) -> int:
    return int(lib().jo_logid_checksum(index, term))


def peerid_checksum(ip: str, port: int, idx: int = 0) -> int:
    return int(lib().jo_peerid_checksum(ip.encode("latin-1"), port, idx))


def logentry_checksum(etype: int, index: int, term: int, peer_xor: int, data: bytes | None) -> int:
    b = b"" if data is None else bytes(data)
    return int(lib().jo_logentry_checksum(etype, index, term, peer_xor, C.c_char_p(b), len(b)))


def logentry_checksum_batch(etype, index, term, peer_xor, payload, offsets, expected=None,
                            has=None):
    etype = np.ascontiguousarray(etype, dtype=np.uint8)
    index = np.ascontiguousarray(index, dtype=np.int64)
    term = np.ascontiguousarray(term, dtype=np.int64)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    if payload.size == 0:
        payload = np.zeros(1, dtype=np.uint8)
    n = len(offsets) - 1
    px = None if peer_xor is None else np.ascontiguousarray(peer_xor, dtype=np.uint64)
    ex = None if expected is None else np.ascontiguousarray(expected, dtype=np.uint64)
    hs = None if has is None else np.ascontiguousarray(has, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint64)
    corrupt = np.zeros(n, dtype=np.uint8) if ex is not None else None
    lib().jo_logentry_checksum_batch(etype, index, term, _ptr(px), payload, offsets, n, out,
                                     _ptr(ex), _ptr(hs), _ptr(corrupt))
    return out if corrupt is None else (out, corrupt)


def append_entries_verify(req_off, prev_log_index, term, etype, data_len, checksum, data,
                          has_checksum=None, peer_xor=None):
    """NodeImpl.handleAppendEntriesRequest's receive loop (NodeImpl.java:1766-1792) for a
    batch of requests; returns (checksum_out, corrupt, first_corrupt)."""
    ro = np.ascontiguousarray(req_off, np.uint32)
    prev = np.ascontiguousarray(prev_log_index, np.int64)
    term = np.ascontiguousarray(term, np.int64)
    et = np.ascontiguousarray(etype, np.uint8)
    dl = np.ascontiguousarray(data_len, np.int64)
    ck = np.ascontiguousarray(checksum, np.uint64)
    hs = None if has_checksum is None else np.ascontiguousarray(has_checksum, np.uint8)
    px = None if peer_xor is None else np.ascontiguousarray(peer_xor, np.uint64)
    d = np.ascontiguousarray(data, np.uint8) if data is not None and len(data) else np.zeros(1, np.uint8)
    N, R = len(term), len(prev)
    out = np.zeros(N, np.uint64)
    cor = np.zeros(N, np.uint8)
    first = np.zeros(R, np.int32)
    lib().jo_append_entries_verify(R, _ptr(ro), _ptr(prev), _ptr(term), _ptr(et), _ptr(dl),
                                   _ptr(px), _ptr(ck), _ptr(hs), _ptr(d), _ptr(out), _ptr(cor),
                                   _ptr(first))
    return out, cor, first


def lease_check(last_rpc_ts, conf, self_slot, now_ms, lease_timeout_ms, lease_start):
    """NodeImpl.handleStepDownTimeout -> checkDeadNodes0 per group (NodeImpl.java:1970-2016)."""
    ts = np.ascontiguousarray(last_rpc_ts, np.int64)
    P, G = ts.shape
    conf = np.ascontiguousarray(conf, np.uint64)
    ss = np.ascontiguousarray(self_slot, np.uint8)
    lead = np.array(lease_start, dtype=np.int64, copy=True)
    ok = np.zeros(G, np.uint8)
    dead = np.zeros(G, np.uint16)
    lib().jo_lease_check(G, P, _ptr(ts), _ptr(conf), _ptr(ss), now_ms, lease_timeout_ms,
                         _ptr(ok), _ptr(lead), _ptr(dead))
    return ok, lead, dead


READINDEX_PENDING, READINDEX_SUCCESS, READINDEX_FAILURE = 0, 1, 2


def readindex_quorum(conf, self_slot, order, ok_mask, P):
    """NodeImpl.readLeader's ReadOnlySafe heartbeat round per group (NodeImpl.java:1246-1396):
    the verdict of ReadIndexHeartbeatResponseClosure over the responses so far."""
    conf = np.ascontiguousarray(conf, np.uint64)
    ss = np.ascontiguousarray(self_slot, np.uint8)
    order = np.ascontiguousarray(order, np.uint64)
    okm = np.ascontiguousarray(ok_mask, np.uint16)
    G = len(conf)
    res = np.zeros(G, np.uint8)
    lib().jo_readindex_quorum(G, P, _ptr(conf), _ptr(ss), _ptr(order), _ptr(okm), _ptr(res))
    return res


FAN_NONE, FAN_APPLY, FAN_SKIP, FAN_INVALID = 0, 1, 2, 3


def commit_fanout_replay(seq_off, seq, last_applied, cq_first, cq_size):
    """FSMCallerImpl.doCommitted per onCommitted call (FSMCallerImpl.java:462-482) over a
    ClosureQueueImpl (ClosureQueueImpl.java:113-142), call by call.  Returns
    (status u8[G], first_closure i64[G], last_applied, cq_first, cq_size, popped_total)."""
    so = np.ascontiguousarray(seq_off, np.uint64)
    G = len(so) - 1
    sq = np.ascontiguousarray(seq, np.int64)
    if sq.size == 0:
        sq = np.zeros(1, np.int64)
    la = np.array(last_applied, dtype=np.int64, copy=True)
    cf = np.array(cq_first, dtype=np.int64, copy=True)
    cs = np.array(cq_size, dtype=np.int64, copy=True)
    fc = np.zeros(G, np.int64)
    st = np.zeros(G, np.uint8)
    n = lib().jo_commit_fanout_replay(G, _ptr(so), _ptr(sq), _ptr(la), _ptr(cf), _ptr(cs),
                                      _ptr(fc), _ptr(st))
    return st, fc, la, cf, cs, int(n)


# ------------------------------------------------------- V2 codec ------------

V2_OK, V2_NULL, V2_V1, V2_PEER_NONCANON, V2_PEER_THROWS = 0, 1, 2, 3, 4
V2_HEADER = bytes([0xBB, 0xD2, 0x01, 0, 0, 0])  # LogEntryV2CodecFactory.java:52-60


def pb_varint(v: int) -> bytes:
    """protobuf varint of a (two's complement, 64-bit) integer."""
    v &= M64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def pb_field(num: int, wire: int, payload: bytes) -> bytes:
    return pb_varint((num << 3) | wire) + payload


def v2_encode(etype: int, index: int, term: int, peers=(), old_peers=(), learners=(),
              old_learners=(), checksum=None, data: bytes | None = b"") -> bytes:
    """V2Encoder.encode (JC/entity/codec/v2/V2Encoder.java:76-130): header + PBLogEntry in
    the generated writeTo order (v2/LogOutter.java:518-546): type 1, term 2, index 3,
    peers 4, old_peers 5, data 6 (always set, EMPTY for null), checksum 7 (if set),
    learners 8, old_learners 9.  Peers are their toString() bytes (latin-1)."""
    b = bytearray(V2_HEADER)
    b += pb_field(1, 0, pb_varint(etype))
    b += pb_field(2, 0, pb_varint(term))
    b += pb_field(3, 0, pb_varint(index))
    for num, lst in ((4, peers), (5, old_peers)):
        for p in lst:
            pb = p.encode("latin-1") if isinstance(p, str) else bytes(p)
            b += pb_field(num, 2, pb_varint(len(pb)) + pb)
    d = data or b""
    b += pb_field(6, 2, pb_varint(len(d)) + d)
    if checksum is not None:
        b += pb_field(7, 0, pb_varint(checksum))
    for num, lst in ((8, learners), (9, old_learners)):
        for p in lst:
            pb = p.encode("latin-1") if isinstance(p, str) else bytes(p)
            b += pb_field(num, 2, pb_varint(len(pb)) + pb)
    return bytes(b)


def v2_peer_checksum(s: bytes):
    """(checksum, kind) of JRaftUtils.getPeerId(s).checksum(); kind 0 canonical, 1 re-rendered,
    2 throws."""
    k = C.c_int(0)
    v = lib().jo_v2_peer_checksum(bytes(s), len(s), C.byref(k))
    return int(v), k.value


def v2_decode_batch(records: np.ndarray, offsets: np.ndarray) -> dict:
    """AutoDetectDecoder/V2Decoder + LogEntry.isCorrupted per record (jo_v2_decode_batch)."""
    rec = np.ascontiguousarray(records, np.uint8)
    if rec.size == 0:
        rec = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(offsets, np.uint64)
    n = len(off) - 1
    o = {k: np.zeros(n, t) for k, t in (
        ("status", np.uint8), ("type", np.uint8), ("index", np.int64), ("term", np.int64),
        ("stored", np.uint64), ("has_checksum", np.uint8), ("data_off", np.uint64),
        ("data_len", np.uint64), ("peer_counts", np.uint32), ("computed", np.uint64),
        ("corrupt", np.uint8))}
    lib().jo_v2_decode_batch(_ptr(rec), _ptr(off), n, *[_ptr(o[k]) for k in (
        "status", "type", "index", "term", "stored", "has_checksum", "data_off", "data_len",
        "peer_counts", "computed", "corrupt")])
    return o


# ------------------------------------------------- pure-Python cross-checks --

def py_table() -> list[int]:
    """Table entries as the doc comment of JC/util/CRC64.java:27-40 defines them."""
    t = []
    for i in range(256):
        c = i << 56
        for _ in range(8):
            c = ((c << 1) ^ POLY) & M64 if c >> 63 else (c << 1) & M64
        t.append(c)
    return t


_PY_T = None


def py_crc64(data: bytes, crc: int = 0) -> int:
    """CRC64.update(byte) loop (JC/util/CRC64.java:100-110), pure Python, small inputs only."""
    global _PY_T
    if _PY_T is None:
        _PY_T = py_table()
    for b in bytes(data):
        crc = _PY_T[((crc >> 56) ^ b) & 0xFF] ^ ((crc << 8) & M64)
    return crc


def py_logid_checksum(index: int, term: int) -> int:
    return py_crc64((index & M64).to_bytes(8, "big") + (term & M64).to_bytes(8, "big"))


def py_peer_string(ip: str, port: int, idx: int = 0) -> str:
    """PeerId.toString (JC/entity/PeerId.java:135-144)."""
    s = f"{ip}:{port}"
    return s + f":{idx}" if idx != 0 else s


def py_peerid_checksum(ip: str, port: int, idx: int = 0) -> int:
    return py_crc64(py_peer_string(ip, port, idx).encode("latin-1"))


# --------------------------------------------------------------- BallotBox --

class BallotBox:
    """ctypes handle on the C restatement of JC/core/BallotBox.java.

    Peers are small integer ids (PeerId.equals == id equality).  Return codes
    follow the reference: bool, or the exception it would throw.
    """

    def __init__(self):
        self._h = lib().jo_bb_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().jo_bb_free(self._h)
            self._h = None

    @property
    def last_committed_index(self):
        return lib().jo_bb_last_committed_index(self._h)

    @property
    def pending_index(self):
        return lib().jo_bb_pending_index(self._h)

    @property
    def queue_size(self):
        return lib().jo_bb_queue_size(self._h)

    @property
    def on_committed_calls(self):
        return lib().jo_bb_on_committed_calls(self._h)

    @property
    def on_committed_last(self):
        return lib().jo_bb_on_committed_last(self._h)

    def commit_at(self, first, last, peer):
        rc = lib().jo_bb_commit_at(self._h, first, last, peer)
        if rc == AIOOBE:
            raise IndexError("ArrayIndexOutOfBoundsException")
        return bool(rc)

    def clear_pending_tasks(self):
        lib().jo_bb_clear_pending_tasks(self._h)

    def reset_pending_index(self, n):
        return bool(lib().jo_bb_reset_pending_index(self._h, n))

    def append_pending_task(self, conf, old_conf=None):
        c = None if conf is None else np.ascontiguousarray(conf, dtype=np.int32)
        o = None if old_conf is None else np.ascontiguousarray(old_conf, dtype=np.int32)
        return bool(lib().jo_bb_append_pending_task(
            self._h, _ptr(c), -1 if c is None else len(c), _ptr(o), -1 if o is None else len(o)))

    def set_last_committed_index(self, idx):
        rc = lib().jo_bb_set_last_committed_index(self._h, idx)
        if rc == IAE:
            raise ValueError("IllegalArgumentException")
        return bool(rc)


def quorum_epoch_replay(match, pending_index, last_appended, last_committed, conf,
                        run_off=None, run_start=None, run_conf=None, chunk=1024):
    """Replay one epoch of a group batch through real BallotBoxes (see jraft_oracle.h).

    Returns (committed[G] int64, status[G] uint8, grants executed)."""
    match = np.ascontiguousarray(match, dtype=np.int64)
    P, G = match.shape
    pending_index = np.ascontiguousarray(pending_index, dtype=np.int64)
    last_appended = np.ascontiguousarray(last_appended, dtype=np.int64)
    last_committed = np.ascontiguousarray(last_committed, dtype=np.int64)
    conf_a = None if conf is None else np.ascontiguousarray(conf, dtype=np.uint64)
    ro = None if run_off is None else np.ascontiguousarray(run_off, dtype=np.uint32)
    rs = None if run_start is None else np.ascontiguousarray(run_start, dtype=np.int64)
    rc = None if run_conf is None else np.ascontiguousarray(run_conf, dtype=np.uint64)
    committed = np.zeros(G, dtype=np.int64)
    status = np.zeros(G, dtype=np.uint8)
    grants = lib().jo_quorum_epoch_replay(G, P, match, pending_index, last_appended,
                                          last_committed, _ptr(conf_a), _ptr(ro), _ptr(rs),
                                          _ptr(rc), chunk, committed, status)
    return committed, status, int(grants)
