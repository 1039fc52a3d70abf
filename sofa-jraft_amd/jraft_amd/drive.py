"""ctypes binding of libjraft_drive.so (sofa-jraft_amd/host/jraft_drive.cpp): a multi-Raft
load driver that replays an epoch series through the C++ host mirror's BallotBox API over
the resident device table, one GroupBatch::flush() per epoch."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib

# (JRAFT_AMD_AB_DRIVE: a variant build's libjraft_drive.so, for tools/gpu_check.sh `dab` A/B
# runs only -- the product path never sets it)
DRIVE_PATH = os.environ.get("JRAFT_AMD_AB_DRIVE") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libjraft_drive.so")
# records: every 8-B update record uploaded (pack records + acks); acks: those written at call
# time as order-free JRQ_ACK records (include/jrq.h), without a pack pass
STATS = ("api_ms", "pack_ms", "device_ms", "deliver_ms", "flush_ms", "h2d_bytes", "d2h_bytes",
         "states", "records", "changed", "api_calls", "acks", "deliver_apply_ms",
         "deliver_callbacks_ms", "pack_wait_ms", "pack_apply_ms",
         "acks_streamed")
_drv = None


def load():
    global _drv
    if _drv is None:
        _lib.load()  # torch's HIP runtime first (see _lib.load)
        if not os.path.exists(DRIVE_PATH):
            raise FileNotFoundError(f"{DRIVE_PATH} missing: run `make -C sofa-jraft_amd`")
        d = C.CDLL(DRIVE_PATH)
        d.jraft_drive_last_error.restype = C.c_char_p
        d.jraft_drive_epochs.restype = C.c_int
        d.jraft_drive_epochs.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.c_uint32] + [C.c_void_p] * 9
        d.jraft_drive_epochs_sharded.restype = C.c_int
        d.jraft_drive_epochs_sharded.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                                 C.c_uint32, C.c_uint32] + [C.c_void_p] * 9
        d.jraft_drive_latency.restype = C.c_int
        d.jraft_drive_latency.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_double, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_void_p]
        _drv = d
    return _drv


def drive_epochs(device: int, s: dict, threads: int = 1, shards: int = 1):
    """Replay series `s` (workloads.host_series) through BallotBox, each epoch's calls made by
    `threads` threads (contiguous group slices); returns (committed [K][G] after each flush,
    stats dict of per-epoch arrays named by STATS).  shards > 1: the groups over that many
    engines on `device` (ShardedGroupBatch), committed read from the published node-wide
    snapshot (checked against every BallotBox inside the driver)."""
    d = load()
    K, P, G = s["match"].shape
    arrs = {k: np.ascontiguousarray(s[k]) for k in ("pending_index", "last_committed", "conf_a",
                                                    "conf_b", "switch_at", "last_appended",
                                                    "match")}
    out = np.zeros((K, G), np.int64)
    stats = np.zeros((K, len(STATS)), np.float64)
    ptr = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    rc = d.jraft_drive_epochs_sharded(device, shards, G, P, K, threads, ptr(arrs["pending_index"]),
                                      ptr(arrs["last_committed"]), ptr(arrs["conf_a"]), ptr(arrs["conf_b"]),
                                      ptr(arrs["switch_at"]), ptr(arrs["last_appended"]), ptr(arrs["match"]),
                                      ptr(out), ptr(stats))
    if rc != 0:
        raise RuntimeError("jraft_drive_epochs: " + (d.jraft_drive_last_error() or b"").decode())
    return out, {k: stats[:, i] for i, k in enumerate(STATS)}


LATENCY = ("commits", "entries", "acks", "seconds", "flushes", "p50_us", "p90_us", "p99_us",
           "p999_us", "max_us", "samples", "producer_duty")


def drive_latency(device: int, groups: int, peers: int, threads: int, seconds: float,
                  max_delay_us: int, max_dirty: int, flush_threads: int = 0, pass_us: int = 0) -> dict:
    """Steady load through BallotBox with the background flusher (GroupBatch::startFlusher,
    FlushPolicy{max_delay_us, max_dirty}): `threads` producers append one entry per group and
    every peer acks it, flush() runs on `flush_threads` threads (0 = its default); returns
    counts and the ack -> onCommitted latency quantiles (us).  pass_us > 0 paces each producer
    to one pass over its groups per pass_us."""
    d = load()
    out = np.zeros(len(LATENCY), np.float64)
    rc = d.jraft_drive_latency(device, groups, peers, threads, flush_threads, seconds,
                               max_delay_us, max_dirty, pass_us, C.c_void_p(out.ctypes.data))
    if rc != 0:
        raise RuntimeError("jraft_drive_latency: " + (d.jraft_drive_last_error() or b"").decode())
    return dict(zip(LATENCY, out.tolist()))
