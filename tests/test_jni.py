"""The JNI binding in source (jni/, VERDICT r05 missing #2).

CPU: the plain-C core compiles with -Wall -Wextra -Werror against include/jrq.h and links
against libjrq.so; jrq_jni.c type-checks against the JNI declarations it uses; a header whose
signatures drift from the glue makes that build fail; every host entry point a JNI host needs
has a core function and a JNIEXPORT.  GPU: the core, called through ctypes with raw addresses
(as the JNIEXPORTs call it with GetDirectBufferAddress), runs the stateless tiled epoch, the
resident table (update, gathered update, epoch) and LogEntry checksums bit-exactly against the
oracle (BallotBox.java:96-139, LogEntry.java:88-108).
"""
import ctypes as C
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from jraft_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "jni")
CORE_SO = os.path.join(JNI, "_build", "libjrq_jni_core.so")

# host-side jrq.h entry points a JNI host does not bind, and why
NOT_BOUND = {
    "jrq_get_stream", "jrq_set_stream",  # HIP stream handles: device-side hosts only
    "jrq_debug_set",                     # test / A-B hooks
    "jrq_table_slices", "jrq_table_view_get", "jrq_table_copy",  # _dev-side table views
    "jrq_rccl_get_unique_id", "jrq_rccl_init", "jrq_rccl_nranks",  # multi-process C++ / Python hosts
}


def _decls(path):
    text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    return set(re.findall(r"\b(jrq_[a-z0-9_]+)\s*\(", text))


def test_core_builds_strict_and_glue_typechecks():
    r = subprocess.run(["make", "-s", "-B", "-C", JNI, "check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(CORE_SO)


def test_header_drift_breaks_the_core(tmp_path):
    """A signature change in include/jrq.h that the glue does not follow fails the strict build."""
    inc = tmp_path / "include"
    inc.mkdir()
    h = open(os.path.join(ROOT, "include", "jrq.h")).read()
    drifted = h.replace("int jrq_crc64_batch(jrq_engine *e, const uint8_t *payload, const uint64_t *offsets,",
                        "int jrq_crc64_batch(jrq_engine *e, const uint8_t *payload, const uint32_t *offsets,")
    assert drifted != h
    (inc / "jrq.h").write_text(drifted)
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-pedantic",
                        "-I" + str(inc), os.path.join(JNI, "jrq_jni_core.c")],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "jrq_crc64_batch" in r.stderr


def test_every_host_entry_point_is_bound():
    header = _decls(_lib.HEADER_PATH)
    host = {f for f in header if not f.endswith("_dev")} - NOT_BOUND
    core = _decls(os.path.join(JNI, "jrq_jni_core.h"))
    core_src = open(os.path.join(JNI, "jrq_jni_core.c")).read()
    missing = sorted(f for f in host if "jrq_jni_" + f[len("jrq_"):] not in core)
    assert not missing, f"jrq.h host entry points without a JNI core function: {missing}"
    # each core function calls its entry point
    for f in host:
        body = core_src.split("jrq_jni_" + f[len("jrq_"):] + "(", 1)[1].split("\n}\n", 1)[0]
        assert f + "(" in body, f
    # each core function has a JNIEXPORT calling it
    glue = open(os.path.join(JNI, "jrq_jni.c")).read()
    uncalled = sorted(c for c in core if c + "(" not in glue)
    assert not uncalled, f"core functions no JNIEXPORT calls: {uncalled}"
    assert glue.count("JNIEXPORT") >= len(core)


def test_negative_java_counts_are_refused_without_a_call():
    L = C.CDLL(CORE_SO)
    L.jrq_jni_crc64_batch.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_int64]
    assert L.jrq_jni_crc64_batch(0, 0, 0, -1, 0) == -1  # JRQ_E_INVALID before libjrq is entered
    L.jrq_jni_table_update_gather.argtypes = [C.c_int64, C.c_int32] + [C.c_int64] * 4
    assert L.jrq_jni_table_update_gather(0, 65, 0, 0, 0, 0) == -1
    L.jrq_jni_build_id.restype = C.c_char_p
    from jraft_amd._srcsha import src_sha
    assert L.jrq_jni_build_id().decode() == src_sha()


def test_jni_build_skips_without_jdk():
    if os.environ.get("JAVA_HOME") or shutil.which("javac"):
        pytest.skip("a JDK is present")
    r = subprocess.run(["make", "-s", "-C", JNI, "jni"], capture_output=True, text=True)
    assert r.returncode == 0 and "skipped" in r.stdout


def _core():
    L = C.CDLL(CORE_SO)
    L.jrq_jni_create.restype = C.c_int64
    L.jrq_jni_create.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int64]
    L.jrq_jni_destroy.argtypes = [C.c_int64]
    L.jrq_jni_last_error.restype = C.c_char_p
    L.jrq_jni_last_error.argtypes = [C.c_int64]
    L.jrq_jni_quorum_epoch_tiles.argtypes = ([C.c_int64, C.c_int64, C.c_int32] + [C.c_int64] * 3
                                             + [C.c_int32, C.c_int64, C.c_int64])
    L.jrq_jni_quorum_epoch.argtypes = ([C.c_int64] * 9 + [C.c_int32] * 3 + [C.c_int64] * 2)
    L.jrq_jni_table_create.restype = C.c_int64
    L.jrq_jni_table_create.argtypes = [C.c_int64, C.c_int32, C.c_int32, C.c_int64]
    L.jrq_jni_table_destroy.argtypes = [C.c_int64]
    L.jrq_jni_table_update.argtypes = [C.c_int64, C.c_int64, C.c_int32, C.c_int64, C.c_int32]
    L.jrq_jni_table_update_gather.argtypes = [C.c_int64, C.c_int32] + [C.c_int64] * 4
    L.jrq_jni_table_epoch.argtypes = [C.c_int64, C.c_int64, C.c_int64]
    L.jrq_jni_table_check.argtypes = [C.c_int64]
    L.jrq_jni_logentry_checksum_batch.argtypes = ([C.c_int64] * 7 + [C.c_int32] + [C.c_int64] * 4)
    return L


def _a(x):
    return 0 if x is None else x.ctypes.data


@pytest.mark.gpu
def test_jni_core_on_gpu(oracle):
    from jraft_amd import Table
    from jraft_amd import workloads as W
    L = _core()
    err = np.zeros(1, np.int32)
    G, P = 4096, 5
    eng = L.jrq_jni_create(0, G, P, _a(err))
    assert eng and err[0] == 0, L.jrq_jni_last_error(0)
    tables = []
    try:
        b = W.quorum_batch("C3", groups=G)
        ce, se, _ = oracle.quorum_epoch_replay(b["match"], b["pending_index"], b["last_appended"],
                                               b["last_committed"], b["conf"], chunk=1024)
        # the stateless contract: one buffer of tiles
        tiles = np.ascontiguousarray(W.to_tiles(b["match"], b["pending_index"], b["last_appended"],
                                                b["last_committed"], b["conf"]))
        c = np.empty(G, np.int64)
        s = np.empty(G, np.uint8)
        assert L.jrq_jni_quorum_epoch_tiles(eng, _a(tiles), P, 0, 0, 0, G, _a(c), _a(s)) == 0
        np.testing.assert_array_equal(c, ce)
        np.testing.assert_array_equal(s, se)
        # rows: P rows of G longs in one buffer
        m = np.ascontiguousarray(b["match"])
        c2 = np.empty(G, np.int64)
        s2 = np.empty(G, np.uint8)
        assert L.jrq_jni_quorum_epoch(eng, _a(m), _a(b["pending_index"]), _a(b["last_appended"]),
                                      _a(b["last_committed"]), _a(b["conf"]), 0, 0, 0, P, 0, G,
                                      _a(c2), _a(s2)) == 0
        np.testing.assert_array_equal(c2, ce)
        # the resident table, once with one update and once with the update in two parts
        pi, lc = b["pending_index"], b["last_committed"]
        st = Table.states(G)
        st["group"] = np.arange(G)
        st["num_runs"] = 1
        st["flags"] = _lib.STATE_RESET_MATCH
        st["pending_index"] = pi
        st["last_appended"] = b["last_appended"]
        st["last_committed"] = lc
        st["run_conf"][:, 0] = b["conf"]
        gs = np.nonzero(pi != 0)[0]
        recs = np.concatenate([_lib.rec(gs, p, np.maximum(b["match"][p, gs] - (pi[gs] - 1), 0))
                               for p in range(P)]).astype(np.uint64)
        for parts in (1, 2):
            t = L.jrq_jni_table_create(eng, G, P, _a(err))
            assert t and err[0] == 0
            tables.append(t)
            if parts == 1:
                assert L.jrq_jni_table_update(t, _a(st), G, _a(recs), len(recs)) == 0
            else:
                # a group's header and its records in the same part
                lo = st[: G // 2]
                hi = st[G // 2:]
                grp = (recs >> np.uint64(5)) & np.uint64((1 << 27) - 1)
                rlo = np.ascontiguousarray(recs[grp < G // 2])
                rhi = np.ascontiguousarray(recs[grp >= G // 2])
                sl, sh = np.ascontiguousarray(lo), np.ascontiguousarray(hi)
                sa = np.array([_a(sl), _a(sh)], np.int64)
                ra = np.array([_a(rlo), _a(rhi)], np.int64)
                ns = np.array([len(sl), len(sh)], np.int32)
                nr = np.array([len(rlo), len(rhi)], np.int32)
                assert L.jrq_jni_table_update_gather(t, 2, _a(sa), _a(ns), _a(ra), _a(nr)) == 0
            changed = np.zeros(G, np.uint64)
            n = L.jrq_jni_table_epoch(t, _a(changed), 0)
            assert n >= 0, L.jrq_jni_last_error(eng)
            assert L.jrq_jni_table_check(t) == 0
            w = changed[:n]
            g = (w & np.uint64(0xFFFFFFFF)).astype(np.int64)
            d = (w >> np.uint64(32)).astype(np.int64)
            got = lc.copy()
            got[g] = pi[g] - 1 + d
            np.testing.assert_array_equal(got, ce)
        # LogEntry.checksum over ragged entries
        offs = W.ragged_offsets(3, 2048, 3000)
        payload = W.random_bytes(3, int(offs[-1]))
        nE = len(offs) - 1
        et = np.full(nE, 2, np.uint8)
        idx = np.arange(1, nE + 1, dtype=np.int64)
        term = np.full(nE, 7, np.int64)
        out = np.empty(nE, np.uint64)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        assert L.jrq_jni_logentry_checksum_batch(eng, _a(et), _a(idx), _a(term), 0, _a(payload),
                                                 _a(offs), nE, _a(out), 0, 0, 0) == 0
        np.testing.assert_array_equal(out, oracle.logentry_checksum_batch(et, idx, term, None,
                                                                          payload, offs))
    finally:
        for t in tables:
            L.jrq_jni_table_destroy(t)
        L.jrq_jni_destroy(eng)
