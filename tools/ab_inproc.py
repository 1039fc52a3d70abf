#!/usr/bin/env python3
"""A/B of libjrq builds in ONE process (tools only): every variant library is loaded side by
side (ctypes, its own engine on the shared stream), and the legs run interleaved round by
round, so box-to-box and warm-up drift fall on every variant alike.

  python tools/ab_inproc.py NAME=PATH.so[:OPT=V,...] [...]   (OPT: jrq_debug_set options by
  name, e.g. CRC_SEG_BYTES=4096 -> jrq_debug_set(e, JRQ_DBG_CRC_SEG_BYTES, 4096))

Per leg and variant: the median over rounds of (one event pair around `reps` back-to-back
launches) / reps, and whether the outputs equal the first variant's.  A torch int64 sum over
the C5 payload is timed alongside as the plain-read reference."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def load_variant(path):
    from jraft_amd import _lib
    from jraft_amd import Engine
    lib = C.CDLL(os.path.abspath(path), mode=C.RTLD_LOCAL)
    for name, res, args in _lib.SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is None:  # an older build without this entry point
            continue
        fn.restype = res
        fn.argtypes = args
    e = Engine.__new__(Engine)
    e._L = lib
    err = C.c_int(0)
    h = lib.jrq_create(0, 1 << 20, 16, C.byref(err))
    if not h:
        raise RuntimeError(f"{path}: jrq_create failed {err.value}")
    e._h = C.c_void_p(h)
    e.device = 0
    return e


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    specs = sys.argv[1:] or ["lib=sofa-jraft_amd/lib/libjrq.so"]
    legs_env = os.environ.get("AB_LEGS", "C5,C1,archive,v2").split(",")
    rounds = int(os.environ.get("AB_ROUNDS", "8"))
    reps = int(os.environ.get("AB_REPS", "10"))
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    import jraft_amd._lib as L
    L.load()  # the in-tree lib first: torch's HIP runtime is already the process runtime
    variants = []
    for sp in specs:
        name, _, rest = sp.partition("=")
        path, _, envs = rest.partition(":")
        e = load_variant(path)
        for kv in filter(None, envs.split(",")):  # per-engine overrides (jrq_debug_set)
            k, _, v = kv.partition("=")
            if e._L.jrq_debug_set(e._h, getattr(L, "DBG_" + k), int(v)) != 0:
                raise RuntimeError(f"{name}: jrq_debug_set {k}={v} refused")
        e._L.jrq_set_stream(e._h, C.c_void_p(s.cuda_stream))
        variants.append((name, e))

    def dev_t(a):
        return torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a).to(dev)

    legs = {}
    eb5 = W.entry_batch(64 << 10, 16 << 10, seed=3)
    d5 = {k: dev_t(v) for k, v in eb5.items() if isinstance(v, np.ndarray)}
    n5 = 64 << 10
    exp5 = torch.zeros(n5, dtype=torch.int64, device=dev)
    outs = {}

    def mk_c5(e, o):
        cor = torch.empty(n5, dtype=torch.uint8, device=dev)
        return lambda: e.logentry_checksum_batch_dev(d5["etype"], d5["index"], d5["term"], None,
                                                     d5["payload"], d5["offsets"], o,
                                                     expected=exp5, corrupt=cor)
    if "C5" in legs_env:
        legs["C5"] = (mk_c5, lambda: torch.empty(n5, dtype=torch.int64, device=dev))
    if "C1" in legs_env:
        eb1 = W.entry_batch(1 << 20, 256, seed=5)
        d1 = {k: dev_t(v) for k, v in eb1.items() if isinstance(v, np.ndarray)}
        legs["C1"] = (lambda e, o: (lambda: e.logentry_checksum_batch_dev(
            d1["etype"], d1["index"], d1["term"], None, d1["payload"], d1["offsets"], o)),
            lambda: torch.empty(1 << 20, dtype=torch.int64, device=dev))
    if "C3" in legs_env:  # the headline: C3 epochs (pair kernel) over 6 rotating inputs
        c3 = []
        for k in range(6):
            b = W.quorum_batch("C3", seed=(W.SEED_BASE ^ 3) + 7919 * k)
            c3.append({kk: dev_t(v) for kk, v in b.items()})
        c3s = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
        def mk_c3(e, o):
            cnt = [0]  # per variant: the same buffer sequence for each

            def f():
                t = c3[cnt[0] % 6]
                cnt[0] += 1
                e.quorum_epoch_dev(t["match"], t["pending_index"], t["last_appended"],
                                   t["last_committed"], t["conf"], o, c3s)
            return f
        legs["C3"] = (mk_c3, lambda: torch.empty(1 << 20, dtype=torch.int64, device=dev))
    if "C3T" in legs_env:  # the headline: C3 epochs from tiles over 6 rotating inputs
        c3t = []
        for k in range(6):
            b = W.quorum_batch("C3", seed=(W.SEED_BASE ^ 3) + 7919 * k)
            c3t.append(torch.from_numpy(W.to_tiles(b["match"], b["pending_index"], b["last_appended"],
                                                   b["last_committed"], b["conf"])).to(dev))
        c3ts = torch.empty(1 << 20, dtype=torch.uint8, device=dev)

        def mk_c3t(e, o):
            ls = [e.quorum_epoch_tiles_launcher(t, 5, 1 << 20, o, c3ts) for t in c3t]
            cnt = [0]

            def f():
                ls[cnt[0] % 6]()
                cnt[0] += 1
            return f
        legs["C3T"] = (mk_c3t, lambda: torch.empty(1 << 20, dtype=torch.int64, device=dev))
    if "C3K" in legs_env:  # 8 epochs of C3 per launch (jrq_quorum_epochs_dev)
        sk = W.quorum_epoch_series("C3", 8)
        dk = {kk: dev_t(np.ascontiguousarray(v)) for kk, v in sk.items()}
        skst = torch.empty((8, 1 << 20), dtype=torch.uint8, device=dev)

        def mk_c3k(e, o):
            return lambda: e.quorum_epochs_dev(dk["match"], dk["pending_index"], dk["last_appended"],
                                               dk["last_committed"], dk["conf"], o, skst)
        legs["C3K"] = (mk_c3k, lambda: torch.empty((8, 1 << 20), dtype=torch.int64, device=dev))
    if "C3KT" in legs_env:  # the same 8 epochs of C3 in the tile layout (jrq_quorum_epochs_tiles_dev)
        skt = W.quorum_epoch_series("C3", 8)
        Gt = skt["pending_index"].shape[0]
        tl = torch.from_numpy(np.stack([W.to_tiles(skt["match"][k], skt["pending_index"],
                                                   skt["last_appended"][k], skt["last_committed"],
                                                   skt["conf"]) for k in range(8)])).to(dev)
        sktst = torch.empty((8, Gt), dtype=torch.uint8, device=dev)

        def mk_c3kt(e, o):
            return e.quorum_epochs_tiles_launcher(tl, 5, Gt, o, sktst)
        legs["C3KT"] = (mk_c3kt, lambda: torch.empty((8, Gt), dtype=torch.int64, device=dev))
    for kk_, KE in (("C2K256", 256), ("C2K64", 64)):  # configs[1], KE epochs per launch
        if kk_ not in legs_env:
            continue
        s2 = W.quorum_epoch_series("C2", KE)
        d2 = {kk: dev_t(np.ascontiguousarray(v)) for kk, v in s2.items()}
        G2 = d2["pending_index"].shape[0]
        st2 = torch.empty((KE, G2), dtype=torch.uint8, device=dev)

        def mk_c2k(e, o, d2=d2, st2=st2):
            return lambda: e.quorum_epochs_dev(d2["match"], d2["pending_index"], d2["last_appended"],
                                               d2["last_committed"], d2["conf"], o, st2)
        legs[kk_] = (mk_c2k, lambda KE=KE, G2=G2: torch.empty((KE, G2), dtype=torch.int64, device=dev))
    if "C5f" in legs_env:  # the C5 entries (16 KiB each) through the fixed-size entry point
        def mk_c5f(e, o):
            cor = torch.empty(n5, dtype=torch.uint8, device=dev)
            return lambda: e.logentry_checksum_fixed_dev(d5["etype"], d5["index"], d5["term"], None,
                                                         d5["payload"], 16 << 10, o,
                                                         expected=exp5, corrupt=cor)
        legs["C5f"] = (mk_c5f, lambda: torch.empty(n5, dtype=torch.int64, device=dev))
    if "C1f" in legs_env:  # the same 256-B entries through the fixed-size entry point
        if "C1" not in legs_env:
            eb1 = W.entry_batch(1 << 20, 256, seed=5)
            d1 = {k: dev_t(v) for k, v in eb1.items() if isinstance(v, np.ndarray)}
        legs["C1f"] = (lambda e, o: (lambda: e.logentry_checksum_fixed_dev(
            d1["etype"], d1["index"], d1["term"], None, d1["payload"], 256, o)),
            lambda: torch.empty(1 << 20, dtype=torch.int64, device=dev))
    if "archive" in legs_env:
        tot = int(d5["payload"].numel())
        one = torch.tensor([0, tot], dtype=torch.int64, device=dev)

        def mk_arch(e, o):
            def f():
                o.zero_()
                e.crc64_stream_update_dev(o, d5["payload"], one)
            return f
        legs["archive"] = (mk_arch, lambda: torch.zeros(1, dtype=torch.int64, device=dev))
    if "v2" in legs_env:
        rec_np, lens = W.v2_records(eb5["etype"], eb5["index"], eb5["term"], eb5["payload"],
                                    eb5["offsets"], np.zeros(n5, np.uint64))
        d_rec = torch.from_numpy(rec_np).to(dev)
        d_roff = dev_t(lens)

        def mk_v2(e, o):
            return lambda: e.v2_decode_verify_dev(d_rec, d_roff, o)

        def new_v2():
            return {k: torch.empty(n5, dtype={np.uint8: torch.uint8, np.uint32: torch.int32}.get(t, torch.int64),
                                   device=dev) for k, t in Engine.V2_FIELDS}
        legs["v2"] = (mk_v2, new_v2)

    if "fanout" in legs_env:  # commit fan-out of a C3 epoch, 1M groups (steady state: after the
        # first launch the queues hold nothing at or below the commit, so no group pops)
        bq = W.quorum_batch("C3")
        Gq = bq["pending_index"].shape[0]
        fq = {k: dev_t(np.ascontiguousarray(v)) for k, v in bq.items()}
        fc_c = torch.empty(Gq, dtype=torch.int64, device=dev)
        fc_s = torch.empty(Gq, dtype=torch.uint8, device=dev)
        variants[0][1].quorum_epoch_dev(fq["match"], fq["pending_index"], fq["last_appended"],
                                        fq["last_committed"], fq["conf"], fc_c, fc_s)
        torch.cuda.synchronize()

        def mk_fan(e, o):
            cf = fq["pending_index"].clone()
            cs = (fq["last_appended"] - fq["pending_index"] + 1).clone()
            la = fq["last_committed"].clone()
            st = torch.empty(Gq, dtype=torch.uint8, device=dev)
            lst = torch.empty((Gq + 63) // 64, dtype=torch.int64, device=dev)
            num = torch.zeros(1, dtype=torch.int32, device=dev)
            return lambda: e.commit_fanout_dev(fq["last_committed"], fc_c, la, cf, cs, o, st, lst, num)
        legs["fanout"] = (mk_fan, lambda: torch.empty(Gq, dtype=torch.int64, device=dev))
    if "tick" in legs_env or "lease" in legs_env:  # leader tick over 1M groups x 5 peers
        Gt, Pt = 1 << 20, 5
        rng = np.random.default_rng(5)
        conf_t = dev_t(W.quorum_batch("C3", groups=Gt)["conf"])
        self_t = torch.zeros(Gt, dtype=torch.uint8, device=dev)
        tb = []
        for k in range(6):
            ts = (1 << 40) - rng.integers(0, 1800, (Pt, Gt)).astype(np.int64)
            order = rng.integers(0, 1 << 20, Gt).astype(np.int64)
            okm = rng.integers(0, 1 << 5, Gt).astype(np.int16)
            tb.append((dev_t(ts), dev_t(order), dev_t(okm)))

        def mk_tick(ri):
            def mk(e, o):
                cnt = [0]
                lead = torch.zeros(Gt, dtype=torch.int64, device=dev)
                dead = torch.empty(Gt, dtype=torch.int16, device=dev)
                res = torch.empty(Gt, dtype=torch.uint8, device=dev)

                def f():
                    ts, order, okm = tb[cnt[0] % 6]
                    cnt[0] += 1
                    e.leader_tick_dev(ts, conf_t, self_t, 1 << 40, 900, o, lead, dead,
                                      order if ri else None, okm if ri else None,
                                      res if ri else None)
                return f
            return mk
        if "tick" in legs_env:
            legs["tick"] = (mk_tick(True), lambda: torch.empty(Gt, dtype=torch.uint8, device=dev))
        if "lease" in legs_env:
            legs["lease"] = (mk_tick(False), lambda: torch.empty(Gt, dtype=torch.uint8, device=dev))
    pay64 = d5["payload"].view(torch.int64)
    acc = torch.empty((), dtype=torch.int64, device=dev)
    fns = {}
    needs = {"C1f": "jrq_logentry_checksum_fixed_dev", "C5f": "jrq_logentry_checksum_fixed_dev"}
    for leg, (mk, new_out) in legs.items():
        for name, e in variants:
            if leg in needs and not hasattr(e._L, needs[leg]):
                continue  # an older build without that entry point
            o = new_out()
            outs[(leg, name)] = o
            fns[(leg, name)] = mk(e, o)
    fns[("read", "torch_sum")] = lambda: torch.sum(pay64, dim=0, out=acc)
    times = {k: [] for k in fns}
    for r in range(rounds + 1):
        for k, f in fns.items():
            f()
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                f()
            z.record(s)
            z.synchronize()
            if r > 0:
                times[k].append(a.elapsed_time(z) / reps)
    res = {}
    for (leg, name), t in times.items():
        o = outs.get((leg, name))
        first = next((outs[(leg, v)] for v, _ in variants if (leg, v) in outs), None)
        same = None
        if o is not None:
            if isinstance(o, dict):
                same = all(torch.equal(o[k], first[k]) for k in o)
            else:
                same = bool(torch.equal(o, first))
        res.setdefault(leg, {})[name] = {"ms_median": float(np.median(t)), "ms_min": float(np.min(t)),
                                         "same_as_first": same}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
