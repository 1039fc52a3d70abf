#!/usr/bin/env python3
"""Alternating A/B of host-mirror builds on the GPU box: the C3 drive series (bench.py leg
`drive`) through each variant's libjraft_drive.so (tools/host_ab_build.sh), round-robin in one
process, `--rounds` times; per variant the median over every steady epoch of api / pack / device /
deliver / flush ms, and whether the commits equal the first variant's.  Not part of any product path.

    python tools/drive_ab.py NAME=ab/NAME/libjraft_drive.so ... [--rounds 5] [--epochs 10]

A variant may carry one environment setting (NAME=path:VAR=VALUE).  Each (round, variant) runs in
its own process: the variants' libjraft_drive.so all name their
host library "libjraft_host.so", and one process would bind every drive to the first one loaded.
        [--flush-threads 16,8]   (each variant once per flush-pool size: NAME@16, NAME@8)
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--active", type=float, default=1.0)
    ap.add_argument("--flush-threads", default="", help="comma list of flush-pool sizes to alternate")
    ap.add_argument("--one", default=None, help="(internal) run one variant once, print its stats")
    a = ap.parse_args()
    if a.one is None:
        return orchestrate(a)
    from jraft_amd import _lib, drive
    from jraft_amd import workloads as W
    _lib.load()
    libs = {}
    for v in [x for x in a.variants if x.split("=", 1)[0] == a.one]:
        name, path = v.split("=", 1)
        if ":" in path:  # NAME=path:VAR=VALUE -- the same build under another setting
            path, env = path.split(":", 1)
            k, val = env.split("=", 1)
            os.environ[k] = val
        d = C.CDLL(os.path.abspath(path))
        d.jraft_drive_last_error.restype = C.c_char_p
        d.jraft_drive_epochs.restype = C.c_int
        d.jraft_drive_epochs.argtypes = [C.c_int] + [C.c_uint32] * 4 + [C.c_void_p] * 9
        for ft in (a.flush_threads.split(",") if a.flush_threads else [""]):
            libs[f"{name}@{ft}" if ft else name] = (d, ft)
    s = W.host_series("C3", a.epochs, groups=a.groups, joint_frac=0.01, active=a.active)
    K, P, G = s["match"].shape
    arrs = {k: np.ascontiguousarray(s[k]) for k in ("pending_index", "last_committed", "conf_a",
                                                    "conf_b", "switch_at", "last_appended", "match")}
    p = lambda x: C.c_void_p(x.ctypes.data)  # noqa: E731
    import hashlib
    for n, (d, ft) in libs.items():
        if ft:
            os.environ["JRAFT_DRIVE_FLUSH_THREADS"] = ft
        out = np.zeros((K, G), np.int64)
        st = np.zeros((K, len(drive.STATS)), np.float64)
        rc = d.jraft_drive_epochs(0, G, P, K, a.threads, p(arrs["pending_index"]), p(arrs["last_committed"]),
                                  p(arrs["conf_a"]), p(arrs["conf_b"]), p(arrs["switch_at"]),
                                  p(arrs["last_appended"]), p(arrs["match"]), p(out), p(st))
        if rc:
            raise SystemExit(f"{n}: " + d.jraft_drive_last_error().decode())
        print("RESULT " + json.dumps({"variant": n, "commits_sha": hashlib.sha256(out.tobytes()).hexdigest(),
                                      "stats": st[1:].tolist()}), flush=True)


def orchestrate(a):
    import subprocess
    from jraft_amd import drive
    runs = [(v.split("=", 1)[0], ft) for v in a.variants
            for ft in (a.flush_threads.split(",") if a.flush_threads else [""])]
    names = [f"{n}@{ft}" if ft else n for n, ft in runs]
    per = {n: [] for n in names}
    sha = {}
    for r in range(a.rounds):
        for (v, ft), n in zip(runs, names):
            cmd = [sys.executable, os.path.abspath(__file__), *a.variants, "--one", v, "--epochs", str(a.epochs),
                   "--threads", str(a.threads), "--groups", str(a.groups), "--active", str(a.active)]
            if ft:
                cmd += ["--flush-threads", ft]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            got = [l for l in out.stdout.splitlines() if l.startswith("RESULT ")]
            if out.returncode != 0 or not got:
                raise SystemExit(f"{n}: rc={out.returncode}\n{out.stderr[-2000:]}")
            for g in got:
                d = json.loads(g[len("RESULT "):])
                per[d["variant"]].append(np.array(d["stats"]))
                sha.setdefault(d["variant"], set()).add(d["commits_sha"])
            m = per[n][-1]
            print(f"round {r} {n}: flush {np.median(m[:, 4]):.2f} deliver {np.median(m[:, 3]):.2f} "
                  f"api {np.median(m[:, 0]):.2f}", flush=True)
    first = next(iter(sha.values()))
    res = {}
    for n, L in per.items():
        m = np.concatenate(L)
        res[n] = {k: round(float(np.median(m[:, i])), 3) for i, k in enumerate(drive.STATS)
                  if k in ("api_ms", "pack_ms", "device_ms", "deliver_ms", "flush_ms", "deliver_apply_ms",
                           "deliver_callbacks_ms", "pack_wait_ms", "pack_apply_ms", "acks", "acks_streamed")}
        res[n]["same_commits"] = sha[n] == first and len(sha[n]) == 1
    print(json.dumps({"threads": a.threads, "groups": a.groups, "epochs": a.epochs, "rounds": a.rounds,
                      "active": a.active, "process_per_run": True, "median_ms": res}))

if __name__ == "__main__":
    main()
