"""Engine: Python handle on a libjrq.so engine (one per GPU / host thread).

Host-pointer methods take numpy arrays and return numpy arrays (the path a Java
host takes with DirectByteBuffers).  ``*_dev`` methods take device buffers that
expose ``data_ptr()`` (torch tensors on ``cuda:N``) and run asynchronously on the
engine's stream; ``use_stream`` makes the engine launch on a caller's stream.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import GROUP_STATE, GroupBatch, TableView, check



def _host_np(t):
    """numpy copy of a device tensor through page-locked host memory: no pageable memory is
    handed to a HIP copy (the round-4/5 faults)."""
    import torch
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h.numpy()

def _np_ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _dev_ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _c(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def listed_ids(bitmap, G: int) -> np.ndarray:
    """Ascending group ids of the set bits of a jrq_commit_fanout bitmap (bit g&63 of word g>>6)."""
    bits = np.unpackbits(np.ascontiguousarray(bitmap, np.uint64).view(np.uint8), bitorder="little")
    return np.nonzero(bits[:G])[0].astype(np.uint32)


class Engine:
    def __init__(self, device: int = 0, max_groups: int = 1 << 20, max_peers: int = 16):
        self._L = _lib.load()
        err = C.c_int(0)
        h = self._L.jrq_create(device, max_groups, max_peers, C.byref(err))
        if not h:
            raise _lib.JrqError(err.value, (self._L.jrq_last_error(None) or b"").decode())
        self._h = C.c_void_p(h)
        self.device = device

    # ------------------------------------------------------------ lifetime --
    def close(self):
        if getattr(self, "_h", None):
            self._L.jrq_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def stream(self) -> int:
        return int(self._L.jrq_get_stream(self._h) or 0)

    def use_stream(self, stream_handle: int | None):
        """Launch on an external hipStream_t (e.g. a torch.cuda.Stream().cuda_stream).

        None (or 0, the default stream's handle) selects the engine's own stream."""
        check(self._L.jrq_set_stream(self._h, C.c_void_p(stream_handle) if stream_handle else None),
              self._h)

    def synchronize(self):
        check(self._L.jrq_synchronize(self._h), self._h)

    def debug_set(self, option: int, value: int):
        """jrq_debug_set: a test / A-B override (_lib.DBG_*) on this engine only."""
        check(self._L.jrq_debug_set(self._h, option, value), self._h)

    # -------------------------------------------------------------- quorum --
    @staticmethod
    def _batch(ptr, match, pending_index, last_appended, last_committed, conf, run_off, run_start,
               run_conf, num_peers, match_ld, num_runs):
        b = GroupBatch()
        b.match = ptr(match)
        b.pending_index = ptr(pending_index)
        b.last_appended = ptr(last_appended)
        b.last_committed = ptr(last_committed)
        b.conf = ptr(conf)
        b.run_off = ptr(run_off)
        b.run_start = ptr(run_start)
        b.run_conf = ptr(run_conf)
        b.num_peers = num_peers
        b.num_runs = num_runs
        b.match_ld = match_ld
        return b

    def quorum_epoch(self, match, pending_index, last_appended, last_committed, conf=None,
                     run_off=None, run_start=None, run_conf=None):
        """Host variant: numpy in, (committed int64[G], status uint8[G]) out."""
        match = _c(match, np.int64)
        P, G = match.shape
        arrs = dict(match=match, pending_index=_c(pending_index, np.int64),
                    last_appended=_c(last_appended, np.int64),
                    last_committed=_c(last_committed, np.int64), conf=_c(conf, np.uint64),
                    run_off=_c(run_off, np.uint32), run_start=_c(run_start, np.int64),
                    run_conf=_c(run_conf, np.uint64))
        nr = 0 if arrs["run_start"] is None else len(arrs["run_start"])
        b = self._batch(_np_ptr, num_peers=P, match_ld=G, num_runs=nr, **arrs)
        committed = np.zeros(G, dtype=np.int64)
        status = np.zeros(G, dtype=np.uint8)
        check(self._L.jrq_quorum_epoch(self._h, C.byref(b), _np_ptr(committed), _np_ptr(status), G),
              self._h)
        return committed, status

    def quorum_epoch_dev(self, match, pending_index, last_appended, last_committed, conf,
                         committed_out, status_out, run_off=None, run_start=None, run_conf=None):
        """Device variant: torch tensors (match shape [P, ld]); asynchronous on the engine stream."""
        P = match.shape[0]
        G = pending_index.shape[0]
        b = self._batch(_dev_ptr, match, pending_index, last_appended, last_committed, conf,
                        run_off, run_start, run_conf, num_peers=P, match_ld=match.stride(0),
                        num_runs=0 if run_start is None else run_start.shape[0])
        check(self._L.jrq_quorum_epoch_dev(self._h, C.byref(b), _dev_ptr(committed_out),
                                           _dev_ptr(status_out), G), self._h)

    def quorum_epoch_tiles_launcher(self, tiles, P, G, committed_out, status_out, run_off=None,
                                    run_start=None, run_conf=None):
        """jrq_quorum_epoch_tiles_dev with its arguments resolved once: `tiles` a device tensor
        in the table's tile layout (to_tiles); returns a zero-argument callable."""
        b = _lib.GroupTiles(_dev_ptr(tiles), P, _dev_ptr(run_off), _dev_ptr(run_start), _dev_ptr(run_conf))
        fn, h, ref = self._L.jrq_quorum_epoch_tiles_dev, self._h, C.byref(b)
        co, so = _dev_ptr(committed_out), _dev_ptr(status_out)
        keep = (b, tiles, committed_out, status_out, run_off, run_start, run_conf)

        def launch():
            rc = fn(h, ref, co, so, G)
            if rc:
                check(rc, h)
        launch.keep = keep
        return launch

    def quorum_epoch_tiles(self, tiles, P, G, run_off=None, run_start=None, run_conf=None):
        """Host variant of the tiled epoch (jrq_quorum_epoch_tiles: the JNI binding's stateless
        contract): `tiles` a numpy int64 array in the tile layout (W.to_tiles).  Returns
        (committed int64[G], status uint8[G])."""
        tiles = _c(tiles, np.int64)
        ro, rs, rc_ = _c(run_off, np.uint32), _c(run_start, np.int64), _c(run_conf, np.uint64)
        b = _lib.GroupTiles(_np_ptr(tiles), P, _np_ptr(ro), _np_ptr(rs), _np_ptr(rc_))
        out = np.zeros(G, np.int64)
        st = np.zeros(G, np.uint8)
        check(self._L.jrq_quorum_epoch_tiles(self._h, C.byref(b), _np_ptr(out), _np_ptr(st), G),
              self._h)
        return out, st

    def quorum_epoch_launcher(self, match, pending_index, last_appended, last_committed, conf,
                              committed_out, status_out, run_off=None, run_start=None,
                              run_conf=None):
        """quorum_epoch_dev with its arguments resolved once: returns a zero-argument callable
        that only makes the C call -- the per-epoch host cost of a C / JNI host that keeps its
        jrq_group_batch (bench.py's epoch loop; Python's per-call argument marshalling would
        otherwise outlast a 17 us epoch)."""
        P = match.shape[0]
        G = pending_index.shape[0]
        b = self._batch(_dev_ptr, match, pending_index, last_appended, last_committed, conf,
                        run_off, run_start, run_conf, num_peers=P, match_ld=match.stride(0),
                        num_runs=0 if run_start is None else run_start.shape[0])
        fn, h, ref = self._L.jrq_quorum_epoch_dev, self._h, C.byref(b)
        co, so = _dev_ptr(committed_out), _dev_ptr(status_out)
        keep = (b, match, pending_index, last_appended, last_committed, conf, committed_out,
                status_out, run_off, run_start, run_conf)

        def launch():
            rc = fn(h, ref, co, so, G)
            if rc:
                check(rc, h)
        launch.keep = keep
        return launch

    def quorum_epochs_launcher(self, match, pending_index, last_appended, last_committed, conf,
                               committed_out, status_out, run_off=None, run_start=None,
                               run_conf=None):
        """quorum_epochs_dev with its arguments resolved once (see quorum_epoch_launcher)."""
        K, P = match.shape[0], match.shape[1]
        G = pending_index.shape[0]
        b = self._batch(_dev_ptr, match, pending_index, last_appended, last_committed, conf,
                        run_off, run_start, run_conf, num_peers=P, match_ld=match.stride(1),
                        num_runs=0 if run_start is None else run_start.shape[0])
        fn, h, ref = self._L.jrq_quorum_epochs_dev, self._h, C.byref(b)
        me, le = match.stride(0), last_appended.stride(0)
        co, so = _dev_ptr(committed_out), _dev_ptr(status_out)
        keep = (b, match, pending_index, last_appended, last_committed, conf, committed_out,
                status_out, run_off, run_start, run_conf)

        def launch():
            rc = fn(h, ref, K, me, le, co, so, G)
            if rc:
                check(rc, h)
        launch.keep = keep
        return launch

    def quorum_epochs_dev(self, match, pending_index, last_appended, last_committed, conf,
                          committed_out, status_out, run_off=None, run_start=None, run_conf=None):
        """K epochs in one launch: match [K, P, ld], last_appended [K, G] (torch tensors);
        committed_out / status_out [K, G].  Conf runs (groups flagged CONF_RUNS in conf) hold
        for all K epochs."""
        K, P = match.shape[0], match.shape[1]
        G = pending_index.shape[0]
        b = self._batch(_dev_ptr, match, pending_index, last_appended, last_committed, conf,
                        run_off, run_start, run_conf, num_peers=P, match_ld=match.stride(1),
                        num_runs=0 if run_start is None else run_start.shape[0])
        check(self._L.jrq_quorum_epochs_dev(self._h, C.byref(b), K, match.stride(0),
                                            last_appended.stride(0), _dev_ptr(committed_out),
                                            _dev_ptr(status_out), G), self._h)

    def quorum_epochs_tiles_launcher(self, tiles, P, G, committed_out, status_out, run_off=None,
                                     run_start=None, run_conf=None):
        """jrq_quorum_epochs_tiles_dev with its arguments resolved once: `tiles` a device tensor
        [K, words] (each row one epoch in the tile layout, W.to_tiles); committed_out /
        status_out [K, G]."""
        K = tiles.shape[0]
        b = _lib.GroupTiles(_dev_ptr(tiles), P, _dev_ptr(run_off), _dev_ptr(run_start), _dev_ptr(run_conf))
        fn, h, ref = self._L.jrq_quorum_epochs_tiles_dev, self._h, C.byref(b)
        ld = tiles.stride(0)
        co, so = _dev_ptr(committed_out), _dev_ptr(status_out)
        keep = (b, tiles, committed_out, status_out, run_off, run_start, run_conf)

        def launch():
            rc = fn(h, ref, K, ld, co, so, G)
            if rc:
                check(rc, h)
        launch.keep = keep
        return launch

    # ------------------------------------------------------------ checksum --
    def crc64_batch(self, payload, offsets):
        payload = _c(payload, np.uint8)
        offsets = _c(offsets, np.uint64)
        n = len(offsets) - 1
        out = np.zeros(max(n, 0), dtype=np.uint64)
        if n > 0:
            if payload.size == 0:
                payload = np.zeros(1, np.uint8)
            check(self._L.jrq_crc64_batch(self._h, _np_ptr(payload), _np_ptr(offsets), n,
                                          _np_ptr(out)), self._h)
        return out

    def crc64_batch_dev(self, payload, offsets, out, n=None):
        n = offsets.shape[0] - 1 if n is None else n
        check(self._L.jrq_crc64_batch_dev(self._h, _dev_ptr(payload), _dev_ptr(offsets), n,
                                          _dev_ptr(out)), self._h)

    def crc64_stream_update(self, state, payload, offsets):
        """CRC64.update(chunk) on S streaming Checksums (include/jrq.h); returns the new
        registers (getValue()).  `state` is not modified."""
        offsets = _c(offsets, np.uint64)
        n = len(offsets) - 1
        st = np.array(state, dtype=np.uint64, copy=True)
        if n > 0:
            if st.shape != (n,):
                raise ValueError("state must hold one register per stream")
            payload = _c(payload, np.uint8)
            if payload.size == 0:
                payload = np.zeros(1, np.uint8)
            check(self._L.jrq_crc64_stream_update(self._h, _np_ptr(st), _np_ptr(payload),
                                                  _np_ptr(offsets), n), self._h)
        return st

    def crc64_stream_update_dev(self, state, payload, offsets, n=None):
        n = offsets.shape[0] - 1 if n is None else n
        check(self._L.jrq_crc64_stream_update_dev(self._h, _dev_ptr(state), _dev_ptr(payload),
                                                  _dev_ptr(offsets), n), self._h)

    def logentry_checksum_batch(self, etype, index, term, peer_xor, payload, offsets,
                                expected=None, has=None):
        etype = _c(etype, np.uint8)
        index = _c(index, np.int64)
        term = _c(term, np.int64)
        peer_xor = _c(peer_xor, np.uint64)
        payload = _c(payload, np.uint8)
        if payload.size == 0:
            payload = np.zeros(1, np.uint8)
        offsets = _c(offsets, np.uint64)
        expected = _c(expected, np.uint64)
        has = _c(has, np.uint8)
        n = len(offsets) - 1
        out = np.zeros(n, dtype=np.uint64)
        corrupt = np.zeros(n, dtype=np.uint8) if expected is not None else None
        if n > 0:
            check(self._L.jrq_logentry_checksum_batch(
                self._h, _np_ptr(etype), _np_ptr(index), _np_ptr(term), _np_ptr(peer_xor),
                _np_ptr(payload), _np_ptr(offsets), n, _np_ptr(out), _np_ptr(expected),
                _np_ptr(has), _np_ptr(corrupt)), self._h)
        return out if corrupt is None else (out, corrupt)

    def crc64_fixed_dev(self, payload, entry_bytes, out, n=None):
        """Device variant over N entries of `entry_bytes` each, back to back (no offsets)."""
        n = out.shape[0] if n is None else n
        check(self._L.jrq_crc64_fixed_dev(self._h, _dev_ptr(payload), entry_bytes, n,
                                          _dev_ptr(out)), self._h)

    def logentry_checksum_fixed_dev(self, etype, index, term, peer_xor, payload, entry_bytes, out,
                                    expected=None, has=None, corrupt=None, n=None):
        n = out.shape[0] if n is None else n
        check(self._L.jrq_logentry_checksum_fixed_dev(
            self._h, _dev_ptr(etype), _dev_ptr(index), _dev_ptr(term), _dev_ptr(peer_xor),
            _dev_ptr(payload), entry_bytes, n, _dev_ptr(out), _dev_ptr(expected),
            _dev_ptr(has), _dev_ptr(corrupt)), self._h)

    def logentry_checksum_batch_dev(self, etype, index, term, peer_xor, payload, offsets, out,
                                    expected=None, has=None, corrupt=None, n=None):
        n = offsets.shape[0] - 1 if n is None else n
        check(self._L.jrq_logentry_checksum_batch_dev(
            self._h, _dev_ptr(etype), _dev_ptr(index), _dev_ptr(term), _dev_ptr(peer_xor),
            _dev_ptr(payload), _dev_ptr(offsets), n, _dev_ptr(out), _dev_ptr(expected),
            _dev_ptr(has), _dev_ptr(corrupt)), self._h)

    # ------------------------------------------------------------ lease --
    def lease_check(self, last_rpc_ts, conf, self_slot, now_ms, lease_timeout_ms,
                    lease_start):
        """Host variant: returns (ok uint8[G], lease_start int64[G], dead uint16[G])."""
        ts = _c(last_rpc_ts, np.int64)
        P, G = ts.shape
        conf = _c(conf, np.uint64)
        self_slot = _c(self_slot, np.uint8)
        lead = np.array(lease_start, dtype=np.int64, copy=True)
        ok = np.zeros(G, np.uint8)
        dead = np.zeros(G, np.uint16)
        check(self._L.jrq_lease_check(self._h, _np_ptr(ts), G, P, _np_ptr(conf), _np_ptr(self_slot),
                                      G, now_ms, lease_timeout_ms, _np_ptr(ok), _np_ptr(lead),
                                      _np_ptr(dead)), self._h)
        return ok, lead, dead

    def lease_check_dev(self, last_rpc_ts, conf, self_slot, now_ms, lease_timeout_ms, ok_out,
                        lease_start_inout, dead_out=None):
        P = last_rpc_ts.shape[0]
        G = conf.shape[0]
        check(self._L.jrq_lease_check_dev(self._h, _dev_ptr(last_rpc_ts), last_rpc_ts.stride(0), P,
                                          _dev_ptr(conf), _dev_ptr(self_slot), G, now_ms,
                                          lease_timeout_ms, _dev_ptr(ok_out),
                                          _dev_ptr(lease_start_inout), _dev_ptr(dead_out)), self._h)

    # ------------------------------------------------------ leader tick --
    def leader_tick(self, last_rpc_ts, conf, self_slot, now_ms, lease_timeout_ms, lease_start,
                    order=None, ok_mask=None):
        """Host variant of jrq_leader_tick: the lease check and (with order / ok_mask) the
        ReadIndex round of the same groups in one launch.  Returns (ok, lease_start, dead,
        ri_result or None)."""
        ts = _c(last_rpc_ts, np.int64)
        P, G = ts.shape
        conf = _c(conf, np.uint64)
        self_slot = _c(self_slot, np.uint8)
        lead = np.array(lease_start, dtype=np.int64, copy=True)
        ok = np.zeros(G, np.uint8)
        dead = np.zeros(G, np.uint16)
        order = _c(order, np.uint64)
        ok_mask = _c(ok_mask, np.uint16)
        res = np.zeros(G, np.uint8) if order is not None else None
        check(self._L.jrq_leader_tick(self._h, _np_ptr(ts), G, P, _np_ptr(conf), _np_ptr(self_slot),
                                      G, now_ms, lease_timeout_ms, _np_ptr(ok), _np_ptr(lead),
                                      _np_ptr(dead), _np_ptr(order), _np_ptr(ok_mask),
                                      _np_ptr(res)), self._h)
        return ok, lead, dead, res

    def leader_tick_dev(self, last_rpc_ts, conf, self_slot, now_ms, lease_timeout_ms, ok_out,
                        lease_start_inout, dead_out=None, order=None, ok_mask=None,
                        ri_result_out=None):
        P = last_rpc_ts.shape[0]
        G = conf.shape[0]
        check(self._L.jrq_leader_tick_dev(self._h, _dev_ptr(last_rpc_ts), last_rpc_ts.stride(0), P,
                                          _dev_ptr(conf), _dev_ptr(self_slot), G, now_ms,
                                          lease_timeout_ms, _dev_ptr(ok_out),
                                          _dev_ptr(lease_start_inout), _dev_ptr(dead_out),
                                          _dev_ptr(order), _dev_ptr(ok_mask),
                                          _dev_ptr(ri_result_out)), self._h)

    def leader_tick_launcher(self, last_rpc_ts, conf, self_slot, now_ms, lease_timeout_ms, ok_out,
                             lease_start_inout, dead_out, order, ok_mask, ri_result_out):
        """The same call with its arguments resolved once (a host keeping its buffers): the
        returned function launches one tick (the bench's step loop)."""
        L, h = self._L, self._h
        P = last_rpc_ts.shape[0]
        G = conf.shape[0]
        args = (h, _dev_ptr(last_rpc_ts), last_rpc_ts.stride(0), P, _dev_ptr(conf),
                _dev_ptr(self_slot), G, now_ms, lease_timeout_ms, _dev_ptr(ok_out),
                _dev_ptr(lease_start_inout), _dev_ptr(dead_out), _dev_ptr(order),
                _dev_ptr(ok_mask), _dev_ptr(ri_result_out))
        fn = L.jrq_leader_tick_dev

        def launch():
            rc = fn(*args)
            if rc:
                check(rc, h)
        return launch

    # -------------------------------------------------------- ReadIndex --
    def readindex_quorum(self, conf, self_slot, order, ok_mask, num_peers):
        """Host variant: the ReadIndex heartbeat round's verdict per group (uint8[G],
        READINDEX_PENDING / _SUCCESS / _FAILURE; include/jrq.h jrq_readindex_quorum)."""
        conf = _c(conf, np.uint64)
        G = len(conf)
        self_slot = _c(self_slot, np.uint8)
        order = _c(order, np.uint64)
        ok_mask = _c(ok_mask, np.uint16)
        res = np.zeros(G, np.uint8)
        check(self._L.jrq_readindex_quorum(self._h, _np_ptr(conf), _np_ptr(self_slot),
                                           _np_ptr(order), _np_ptr(ok_mask), num_peers, G,
                                           _np_ptr(res)), self._h)
        return res

    def readindex_launcher(self, conf, self_slot, order, ok_mask, num_peers, result_out):
        """readindex_quorum_dev with its arguments resolved once (the bench's step loop)."""
        h, fn = self._h, self._L.jrq_readindex_quorum_dev
        args = (h, _dev_ptr(conf), _dev_ptr(self_slot), _dev_ptr(order), _dev_ptr(ok_mask),
                num_peers, conf.shape[0], _dev_ptr(result_out))

        def launch():
            rc = fn(*args)
            if rc:
                check(rc, h)
        return launch

    def readindex_quorum_dev(self, conf, self_slot, order, ok_mask, num_peers, result_out):
        G = conf.shape[0]
        check(self._L.jrq_readindex_quorum_dev(self._h, _dev_ptr(conf), _dev_ptr(self_slot),
                                               _dev_ptr(order), _dev_ptr(ok_mask), num_peers, G,
                                               _dev_ptr(result_out)), self._h)

    # ------------------------------------------------- AppendEntries verify --
    def append_entries_verify(self, req_off, prev_log_index, term, etype, data_len, checksum,
                              data, has_checksum=None, peer_xor=None):
        """Host variant: returns (checksum_out uint64[N], corrupt uint8[N], first_corrupt int32[R])."""
        req_off = _c(req_off, np.uint32)
        prev = _c(prev_log_index, np.int64)
        R = len(prev)
        term = _c(term, np.int64)
        N = len(term)
        etype = _c(etype, np.uint8)
        data_len = _c(data_len, np.int64)
        checksum = _c(checksum, np.uint64)
        has = _c(has_checksum, np.uint8)
        px = _c(peer_xor, np.uint64)
        data = _c(data, np.uint8)
        if data is None or data.size == 0:
            data = np.zeros(1, np.uint8)
        out = np.zeros(N, np.uint64)
        cor = np.zeros(N, np.uint8)
        first = np.zeros(R, np.int32)
        check(self._L.jrq_append_entries_verify(
            self._h, R, _np_ptr(req_off), _np_ptr(prev), N, _np_ptr(term), _np_ptr(etype),
            _np_ptr(data_len), _np_ptr(px), _np_ptr(checksum), _np_ptr(has), _np_ptr(data),
            _np_ptr(out), _np_ptr(cor), _np_ptr(first)), self._h)
        return out, cor, first

    def append_entries_verify_dev(self, req_off, prev_log_index, term, etype, data_len, checksum,
                                  data, checksum_out, corrupt_out, first_corrupt_out,
                                  has_checksum=None, peer_xor=None):
        check(self._L.jrq_append_entries_verify_dev(
            self._h, prev_log_index.shape[0], _dev_ptr(req_off), _dev_ptr(prev_log_index),
            term.shape[0], _dev_ptr(term), _dev_ptr(etype), _dev_ptr(data_len),
            _dev_ptr(peer_xor), _dev_ptr(checksum), _dev_ptr(has_checksum), _dev_ptr(data),
            _dev_ptr(checksum_out), _dev_ptr(corrupt_out), _dev_ptr(first_corrupt_out)), self._h)

    # ---------------------------------------------------------- commit fan-out --
    def commit_fanout(self, prev_committed, committed, last_applied, cq_first, cq_size):
        """Host variant: returns (status u8[G], first_closure i64[G], listed u32[n] (ascending
        group ids decoded from the bitmap), cq_first i64[G], cq_size i64[G]) --
        FSMCallerImpl.doCommitted per group."""
        prev = _c(prev_committed, np.int64)
        com = _c(committed, np.int64)
        la = _c(last_applied, np.int64)
        G = len(com)
        cf = np.array(cq_first, dtype=np.int64, copy=True)
        cs = np.array(cq_size, dtype=np.int64, copy=True)
        fc = np.zeros(G, np.int64)
        st = np.zeros(G, np.uint8)
        bitmap = np.zeros(max((G + 63) // 64, 1), np.uint64)
        num = np.zeros(1, np.uint32)
        check(self._L.jrq_commit_fanout(self._h, G, _np_ptr(prev), _np_ptr(com), _np_ptr(la),
                                        _np_ptr(cf), _np_ptr(cs), _np_ptr(fc), _np_ptr(st),
                                        _np_ptr(bitmap), _np_ptr(num)), self._h)
        listed = listed_ids(bitmap, G)
        if len(listed) != int(num[0]):
            raise _lib.JrqError(-6, "listed bitmap / count mismatch")
        return st, fc, listed, cf, cs

    def commit_fanout_dev(self, prev_committed, committed, last_applied, cq_first, cq_size,
                          first_closure_out, status_out, listed_bitmap_out, num_listed_out):
        check(self._L.jrq_commit_fanout_dev(
            self._h, committed.shape[0], _dev_ptr(prev_committed), _dev_ptr(committed),
            _dev_ptr(last_applied), _dev_ptr(cq_first), _dev_ptr(cq_size),
            _dev_ptr(first_closure_out), _dev_ptr(status_out), _dev_ptr(listed_bitmap_out),
            _dev_ptr(num_listed_out)), self._h)

    # --------------------------------------------------- V2 decode + verify --
    V2_FIELDS = (("status", np.uint8), ("type", np.uint8), ("index", np.int64),
                 ("term", np.int64), ("stored", np.uint64), ("has_checksum", np.uint8),
                 ("data_off", np.uint64), ("data_len", np.uint64), ("peer_counts", np.uint32),
                 ("computed", np.uint64), ("corrupt", np.uint8))

    def v2_decode_verify(self, records, offsets):
        """Host variant: dict of per-record arrays (jrq_v2_decode_verify)."""
        rec = _c(records, np.uint8)
        off = _c(offsets, np.uint64)
        n = len(off) - 1
        o = {k: np.zeros(n, t) for k, t in self.V2_FIELDS}
        check(self._L.jrq_v2_decode_verify(self._h, _np_ptr(rec), _np_ptr(off), n,
                                           *[_np_ptr(o[k]) for k, _ in self.V2_FIELDS]), self._h)
        return o

    def v2_decode_verify_dev(self, records, offsets, out: dict, n=None):
        """Device variant: `out` maps the V2_FIELDS names to device tensors."""
        n = offsets.shape[0] - 1 if n is None else n
        check(self._L.jrq_v2_decode_verify_dev(self._h, _dev_ptr(records), _dev_ptr(offsets), n,
                                               *[_dev_ptr(out.get(k)) for k, _ in self.V2_FIELDS]),
              self._h)

    # ---------------------------------------------------------------- RCCL --
    @staticmethod
    def rccl_unique_id() -> bytes:
        L = _lib.load()
        buf = (C.c_uint8 * 128)()
        check(L.jrq_rccl_get_unique_id(buf))
        return bytes(buf)

    def rccl_init(self, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(self._L.jrq_rccl_init(self._h, nranks, rank, buf), self._h)

    def rccl_nranks(self) -> int:
        """Ranks RCCL counts in this engine's communicator (0 before rccl_init)."""
        n = self._L.jrq_rccl_nranks(self._h)
        if n < 0:
            check(n, self._h)
        return n

    def publish_committed_dev(self, local, global_out):
        check(self._L.jrq_publish_committed_dev(self._h, _dev_ptr(local), _dev_ptr(global_out),
                                                local.shape[0]), self._h)


class Table:
    """A resident group table (include/jrq.h jrq_table) on an Engine's device: the BallotBox
    state of G groups x P peer slots kept in HBM, incremental updates, epochs that return only
    the groups whose commit advanced."""

    def __init__(self, engine: Engine, G: int, num_peers: int):
        self._eng = engine
        self._L = engine._L
        err = C.c_int(0)
        h = self._L.jrq_table_create(engine.handle, G, num_peers, C.byref(err))
        if not h:
            raise _lib.JrqError(err.value, (self._L.jrq_last_error(engine.handle) or b"").decode())
        self._h = C.c_void_p(h)
        self.G, self.P = G, num_peers

    def close(self):
        if getattr(self, "_h", None):
            self._L.jrq_table_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def states(n: int) -> np.ndarray:
        """A zeroed array of n jrq_group_state records."""
        return np.zeros(n, dtype=GROUP_STATE)

    def update(self, states=None, recs=None):
        """Host variant: states (GROUP_STATE array) then recs (uint64 JRQ_REC words)."""
        st = None if states is None else np.ascontiguousarray(states, dtype=GROUP_STATE)
        rc = None if recs is None else np.ascontiguousarray(recs, dtype=np.uint64)
        check(self._L.jrq_table_update(self._h, _np_ptr(st), 0 if st is None else len(st),
                                       _np_ptr(rc), 0 if rc is None else len(rc)), self._eng.handle)
        # the host buffers must outlive the asynchronous copies: keep them until the next epoch
        self._keep = (st, rc)

    def update_dev(self, states=None, recs=None, n_states=None, n_recs=None):
        ns = 0 if states is None else (states.numel() // 96 if n_states is None else n_states)
        nr = 0 if recs is None else (recs.numel() if n_recs is None else n_recs)
        check(self._L.jrq_table_update_dev(self._h, _dev_ptr(states), ns, _dev_ptr(recs), nr),
              self._eng.handle)

    def stage_reserve(self, max_states: int, max_recs: int, max_acks: int = 0, max_segments: int = 1):
        """jrq_table_stage_reserve (+ jrq_table_stage_reserve_acks): staging for the streamed
        update (headers, JRQ_REC records, order-free JRQ_ACK segments)."""
        check(self._L.jrq_table_stage_reserve(self._h, max_states, max_recs), self._eng.handle)
        check(self._L.jrq_table_stage_reserve_acks(self._h, max_acks, max_segments), self._eng.handle)
        self._staged = []

    def stage(self, states=None, recs=None):
        st = None if states is None else np.ascontiguousarray(states, dtype=GROUP_STATE)
        rc = None if recs is None else np.ascontiguousarray(recs, dtype=np.uint64)
        check(self._L.jrq_table_stage(self._h, _np_ptr(st), 0 if st is None else len(st),
                                      _np_ptr(rc), 0 if rc is None else len(rc)), self._eng.handle)
        self._staged.append((st, rc))

    def stage_acks(self, stamp: int, acks):
        """One segment of order-free JRQ_ACK records recorded under reset stamp `stamp`."""
        a = np.ascontiguousarray(acks, dtype=np.uint64)
        check(self._L.jrq_table_stage_acks(self._h, stamp, _np_ptr(a), len(a)), self._eng.handle)
        self._staged.append(a)

    def stage_apply(self):
        check(self._L.jrq_table_stage_apply(self._h), self._eng.handle)
        self._keep = self._staged

    def epoch(self, status: bool = False):
        """Host variant: returns (changed uint64[n] as JRQ words, status uint8[G] or None)."""
        out = np.zeros(max(self.G, 1), np.uint64)
        n = C.c_uint32(0)
        st = np.zeros(self.G, np.uint8) if status else None
        check(self._L.jrq_table_epoch(self._h, _np_ptr(out), C.byref(n), _np_ptr(st)),
              self._eng.handle)
        self._keep = None
        return out[: n.value].copy(), st

    def slices(self) -> int:
        """Slices of the device variant's changed list (one per TABLE_SLICE groups)."""
        return int(self._L.jrq_table_slices(self._h))

    def list_buffers(self, device):
        """(changed_out, n_changed_out) device tensors sized for epoch_dev."""
        import torch
        s = self.slices()
        return (torch.empty(s * _lib.TABLE_SLICE, dtype=torch.int64, device=device),
                torch.zeros(s, dtype=torch.int32, device=device))

    def epoch_dev(self, changed_out, n_changed_out, status_out=None):
        """Device variant: changed_out capacity TABLE_SLICE * slices() words, n_changed_out
        int32[slices()] per-slice counts (slice s lists groups [128 s, 128 s + 128) at
        changed_out[128 s ..], see include/jrq.h)."""
        check(self._L.jrq_table_epoch_dev(self._h, _dev_ptr(changed_out), _dev_ptr(n_changed_out),
                                          _dev_ptr(status_out)), self._eng.handle)

    def gather_dev_list(self, changed_out, n_changed_out) -> np.ndarray:
        """Host copy of a device-variant list as the host variant's words (delta << 32 | group),
        slices in order: each slice is a 128-bit map of its listed groups, then their u32
        deltas in group order (include/jrq.h jrq_table_epoch_dev)."""
        return decode_slices(_host_np(changed_out), _host_np(n_changed_out))

    # ------------------------------------- FSMCaller state + fused fan-out (r06) --
    def fsm_update(self, groups, last_applied, cq_first, cq_size):
        """Host variant of jrq_table_fsm_update: n groups' lastAppliedIndex and ClosureQueue
        (firstIndex, size)."""
        g = _c(groups, np.uint32)
        a, f, z = (_c(x, np.int64) for x in (last_applied, cq_first, cq_size))
        check(self._L.jrq_table_fsm_update(self._h, _np_ptr(g), _np_ptr(a), _np_ptr(f), _np_ptr(z), len(g)),
              self._eng.handle)

    def fsm_update_dev(self, groups, last_applied, cq_first, cq_size, n=None):
        n = groups.shape[0] if n is None else n
        check(self._L.jrq_table_fsm_update_dev(self._h, _dev_ptr(groups), _dev_ptr(last_applied),
                                               _dev_ptr(cq_first), _dev_ptr(cq_size), n), self._eng.handle)

    def fsm_read(self):
        """(last_applied, cq_first, cq_size), G int64 each."""
        o = [np.zeros(self.G, np.int64) for _ in range(3)]
        check(self._L.jrq_table_fsm_read(self._h, *[_np_ptr(x) for x in o]), self._eng.handle)
        return tuple(o)

    def epoch_fanout(self):
        """Host variant of jrq_table_epoch_fanout: (changed uint64[n] as JRQ words, fan_first
        int64[n], fan_status uint8[n]) -- the epoch and each listed group's doCommitted /
        popClosureUntil in list order."""
        n0 = max(self.G, 1)
        out = np.zeros(n0, np.uint64)
        ff = np.zeros(n0, np.int64)
        fs = np.zeros(n0, np.uint8)
        n = C.c_uint32(0)
        check(self._L.jrq_table_epoch_fanout(self._h, _np_ptr(out), C.byref(n), _np_ptr(ff), _np_ptr(fs)),
              self._eng.handle)
        self._keep = None
        k = n.value
        return out[:k].copy(), ff[:k].copy(), fs[:k].copy()

    def committed_dev(self, out):
        """Every group's lastCommittedIndex into the device tensor `out` (G int64, group order)."""
        check(self._L.jrq_table_committed_dev(self._h, _dev_ptr(out)), self._eng.handle)

    def fan_buffers(self, device):
        """(fan_first_out, fan_status_out) device tensors sized for epoch_fanout_dev."""
        import torch
        s = self.slices()
        return (torch.empty(s * _lib.TABLE_SLICE, dtype=torch.int64, device=device),
                torch.empty(s * _lib.TABLE_SLICE, dtype=torch.uint8, device=device))

    def epoch_fanout_dev(self, changed_out, n_changed_out, fan_first_out, fan_status_out):
        check(self._L.jrq_table_epoch_fanout_dev(self._h, _dev_ptr(changed_out), _dev_ptr(n_changed_out),
                                                 _dev_ptr(fan_first_out), _dev_ptr(fan_status_out)),
              self._eng.handle)

    def read(self) -> dict:
        G, P = self.G, self.P
        o = dict(pending_index=np.zeros(G, np.int64), last_appended=np.zeros(G, np.int64),
                 last_committed=np.zeros(G, np.int64), match=np.zeros((P, G), np.int64))
        check(self._L.jrq_table_read(self._h, _np_ptr(o["pending_index"]),
                                     _np_ptr(o["last_appended"]), _np_ptr(o["last_committed"]),
                                     _np_ptr(o["match"])), self._eng.handle)
        return o

    def check(self):
        """Raise JrqError if invalid headers / records were skipped since the last check."""
        check(self._L.jrq_table_check(self._h), self._eng.handle)

    def copy_from(self, src: "Table"):
        """Device-side copy of src's whole state (same shape), on this engine's stream."""
        check(self._L.jrq_table_copy(self._h, src._h), self._eng.handle)

    def view(self) -> TableView:
        v = TableView()
        check(self._L.jrq_table_view_get(self._h, C.byref(v)), self._eng.handle)
        return v


def decode_slices(slices, counts, S: int | None = None) -> np.ndarray:
    """jrq_table_epoch_dev's slices (int64 / uint64 words, JRQ_TABLE_SLICE per slice) and
    per-slice counts -> the host list's words (delta << 32 | group), in group order.  (`S`:
    another library build's slice size, for A/B tools.)"""
    S = _lib.TABLE_SLICE if S is None else S
    w = np.ascontiguousarray(slices).view(np.uint64).reshape(-1, S)
    counts = np.asarray(counts).astype(np.int64)
    mw = S // 64  # map words per slice
    bits = np.unpackbits(np.ascontiguousarray(w[:, :mw]).view(np.uint8), axis=1, bitorder="little").astype(bool)
    if not np.array_equal(bits.sum(axis=1), counts[:len(bits)]):
        raise AssertionError("slice maps disagree with the per-slice counts")
    deltas = np.ascontiguousarray(w[:, mw:]).view(np.uint32)  # [slices][2 (S - mw)]
    keep = np.arange(deltas.shape[1])[None, :] < counts[:, None]
    groups = (np.nonzero(bits)[0] * S + np.nonzero(bits)[1]).astype(np.uint64)
    return (deltas[keep].astype(np.uint64) << np.uint64(32)) | groups


def decode_changed(words) -> tuple[np.ndarray, np.ndarray]:
    """(group uint32[n], delta int64[n]) of jrq_table_epoch's output words: the group's new
    lastCommittedIndex = its pendingIndex before the epoch - 1 + delta."""
    w = np.asarray(words, dtype=np.uint64)
    return (w & np.uint64(0xFFFFFFFF)).astype(np.uint32), (w >> np.uint64(32)).astype(np.int64)
