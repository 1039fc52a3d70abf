#!/usr/bin/env python3
"""CPU-only probe of the host mirror's per-call cost: the C3 drive series
(bench.py leg `drive`) replayed through jraft_drive_epochs, linked against the libjrq test double
(tests/cpp/fake_jrq.cpp built with -DFAKE_JRQ_CLOSED_FORM: the table in host memory, decided in
closed form) instead of the GPU library.  The API calls and the flush's pack / deliver passes run
the product host code; only the "device" part is the double's.  Not part of any product path.

    python tools/api_probe.py [--groups N] [--threads 1,8] [--epochs K]
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))
OUT = os.path.join(ROOT, "tools", "_build")
LIB = os.path.join(OUT, "libjraft_drive_fake.so")


def build(flags="-O2 -fno-semantic-interposition", host_src=None):
    os.makedirs(OUT, exist_ok=True)
    srcs = [os.path.join(ROOT, p) for p in ("sofa-jraft_amd/host/jraft_drive.cpp",
                                            "sofa-jraft_amd/host/jraft_host.cpp",
                                            "tests/cpp/fake_jrq.cpp")]
    if host_src:  # an A/B variant of the mirror (it includes "jraft_host.h" from its own dir;
        srcs[1] = host_src  # a jraft_drive.cpp beside it is built instead of the tree's)
        drv = os.path.join(os.path.dirname(host_src), "jraft_drive.cpp")
        if os.path.exists(drv):
            srcs[0] = drv
    ora = os.path.join(OUT, "oracle_probe.o")
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-std=c11", "-c",
                           os.path.join(ROOT, "oracle/jraft_oracle.c"), "-o", ora])
    subprocess.check_call(["g++", *flags.split(), "-std=c++17", "-fPIC", "-shared",
                           "-DFAKE_JRQ_CLOSED_FORM", "-o", LIB, *srcs, ora, "-lpthread"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--threads", default="1,8")
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--active", type=float, default=1.0)
    ap.add_argument("--no-build", action="store_true")
    ap.add_argument("--host-src", default=None, help="a variant of host/jraft_host.cpp to A/B")
    a = ap.parse_args()
    if not a.no_build:
        build(host_src=a.host_src)
    from jraft_amd import workloads as W
    d = C.CDLL(LIB)
    d.jraft_drive_last_error.restype = C.c_char_p
    d.jraft_drive_epochs.restype = C.c_int
    d.jraft_drive_epochs.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32] + [C.c_void_p] * 9
    s = W.host_series("C3", a.epochs, groups=a.groups, joint_frac=0.01, active=a.active)
    K, P, G = s["match"].shape
    arrs = {k: np.ascontiguousarray(s[k]) for k in ("pending_index", "last_committed", "conf_a",
                                                    "conf_b", "switch_at", "last_appended", "match")}
    from jraft_amd.drive import STATS as names
    for T in [int(x) for x in a.threads.split(",")]:
        out = np.zeros((K, G), np.int64)
        st = np.zeros((K, len(names)), np.float64)
        p = lambda x: C.c_void_p(x.ctypes.data)  # noqa: E731
        rc = d.jraft_drive_epochs(0, G, P, K, T, p(arrs["pending_index"]), p(arrs["last_committed"]),
                                  p(arrs["conf_a"]), p(arrs["conf_b"]), p(arrs["switch_at"]),
                                  p(arrs["last_appended"]), p(arrs["match"]), p(out), p(st))
        if rc:
            raise SystemExit(d.jraft_drive_last_error().decode())
        m = st[1:].mean(axis=0)
        r = dict(zip(names, m))
        print(f"threads {T}: api {r['api_ms']:.2f} ms ({r['api_calls'] / 1e6:.2f}M calls, "
              f"{r['api_ms'] * 1e6 * T / r['api_calls']:.1f} ns/call/thread), pack {r['pack_ms']:.2f} ms, "
              f"fake device {r['device_ms']:.2f} ms, deliver {r['deliver_ms']:.2f} ms, "
              f"changed {r['changed']:.0f}; first epoch api {st[0, 0]:.1f} ms flush {st[0, 4]:.1f} ms",
              flush=True)


if __name__ == "__main__":
    main()
