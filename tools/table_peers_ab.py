"""A/B (tools only): the resident table epoch at P peers (1M groups, every group committing),
libjrq builds side by side in one process (tools/ab_inproc.py loading), alternating per round.

  P=9 python tools/table_peers_ab.py old=ab/old/libjrq.so new=ab/new/libjrq.so"""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd")); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch
import ctypes as C
from ab_inproc import load_variant
import jraft_amd._lib as L
from jraft_amd import Table

def main():
    P = int(os.environ.get("P", "9")); G = 1 << 20; NB = 4
    dev = torch.device("cuda:0"); s = torch.cuda.Stream(dev); torch.cuda.set_stream(s)
    L.load()
    rng = np.random.default_rng(1)
    res = {}
    variants = []
    for sp in sys.argv[1:]:
        name, _, path = sp.partition("=")
        e = load_variant(path); e._L.jrq_set_stream(e._h, C.c_void_p(s.cuda_stream)); variants.append((name, e))
    tabs = {}
    for name, e in variants:
        prist, work = [], []
        for k in range(NB):
            r = np.random.default_rng(100 + k)
            st = Table.states(G)
            st["group"] = np.arange(G); st["num_runs"] = 1; st["flags"] = L.STATE_RESET_MATCH
            lc = r.integers(1 << 20, 1 << 30, G)
            st["pending_index"] = L.PI_FOLLOWS_LC; st["last_committed"] = lc
            st["last_appended"] = lc + 64
            peers = np.arange(P, dtype=np.uint64)
            conf = np.uint64(((1 << P) - 1) | ((P // 2 + 1) << 32))
            st["run_conf"][:, 0] = conf
            ff = float(os.environ.get("FLAG_FRAC", "0"))  # groups with a conf change in the window
            if ff > 0:
                fl = r.random(G) < ff
                st["num_runs"] = np.where(fl, 2, 1)
                st["run_start"][:, 1] = np.where(fl, lc + 33, 0)
                st["run_conf"][:, 1] = np.where(fl, np.uint64(((1 << P) - 1) | ((P // 2 + 1) << 32) |
                                                              (0b111 << 16) | (2 << 40)), 0)
            gs = np.arange(G)
            recs = np.concatenate([L.rec(gs, p, r.integers(0, 65, G)) for p in range(P)])
            t = Table(e, G, P); t.update(st, recs); prist.append(t); work.append(Table(e, G, P))
        torch.cuda.synchronize()
        # this build's list slice size (256 before r06, 128 since): from its slice count
        sl = work[0].slices()
        S = 256 if sl == (G + 255) // 256 else 128
        bufs = [(torch.empty(sl * S, dtype=torch.int64, device=dev), torch.zeros(sl, dtype=torch.int32, device=dev))
                for _ in work]
        tabs[name] = (prist, work, bufs, S)
    times = {n: [] for n, _ in variants}
    for rep in range(12):
        for name, _ in variants:
            prist, work, lists, _ = tabs[name]
            for w, t in zip(work, prist): w.copy_from(t)
            a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for i in range(NB): work[i].epoch_dev(*lists[i])
            z.record(s); z.synchronize()
            if rep >= 2: times[name].append(a.elapsed_time(z) / NB * 1e3)
    def lists_of(n):  # (a diagnosis variant may write no list: None)
        try:
            from jraft_amd.engine import decode_slices, _host_np
            return [decode_slices(_host_np(l[0]), _host_np(l[1]), tabs[n][3]) for l in tabs[n][2]]
        except AssertionError:
            return None
    outs = {n: lists_of(n) for n, _ in variants}
    names = [n for n, _ in variants]
    same = {n: outs[n] is not None and all(np.array_equal(np.asarray(a), np.asarray(b))
                                         for a, b in zip(outs[names[0]], outs[n])) for n in names}
    print(json.dumps({"P": P, "flag_frac": os.environ.get("FLAG_FRAC", "0"), "us": {n: float(np.median(t)) for n, t in times.items()},
                      "changed": len(outs[names[0]][0]), "same_as_first": same}))

if __name__ == "__main__":
    main()
