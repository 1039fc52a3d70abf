#!/usr/bin/env python3
"""Per-launch times over a long back-to-back series (tools only): does a kernel slow down
under sustained load, and does a plain streaming read slow down the same way?

  python tools/sustain.py [launches]

Series: C5 LogEntry verify (the CRC rounds + finish kernels), a torch int64 sum over the same
1 GiB payload (read-only stream), then C5 again after 200 ms idle.  Prints the per-launch ms at
a few points of each series and the mean over tenths of it."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def series(s, n, fn):
    import torch
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record(s)
    for i in range(n):
        fn()
        ev[i + 1].record(s)
    ev[-1].synchronize()
    t = np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(n)])
    tenths = [float(x.mean()) for x in np.array_split(t, 10)]
    return {"first": [float(x) for x in t[:5]], "tenths_mean_ms": tenths,
            "min": float(t.min()), "mean": float(t.mean())}


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    e = Engine(0)
    e.use_stream(s.cuda_stream)
    N, eb = 64 << 10, 16 << 10
    b = W.entry_batch(N, eb, seed=3)
    d = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
         for k, v in b.items() if isinstance(v, np.ndarray)}
    out = torch.empty(N, dtype=torch.int64, device=dev)
    exp = torch.zeros(N, dtype=torch.int64, device=dev)
    cor = torch.empty(N, dtype=torch.uint8, device=dev)

    def crc():
        e.logentry_checksum_batch_dev(d["etype"], d["index"], d["term"], None, d["payload"],
                                      d["offsets"], out, expected=exp, corrupt=cor)

    pay64 = d["payload"].view(torch.int64)
    acc = torch.empty((), dtype=torch.int64, device=dev)

    def rd():
        torch.sum(pay64, dim=0, out=acc)

    for _ in range(3):
        crc()
        rd()
    torch.cuda.synchronize()
    res = {"crc": series(s, n, crc)}
    time.sleep(0.2)
    res["torch_sum"] = series(s, n, rd)
    time.sleep(0.2)
    res["crc_after_idle"] = series(s, n, crc)
    res["payload_bytes"] = N * eb
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
