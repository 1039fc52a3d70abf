#!/usr/bin/env python3
"""A/B the CRC64 kernel's segment size in ONE process (interleaved rounds).

Each variant is an engine created with its own JRQ_CRC_SEG_BYTES (0 = automatic);
all variants hash the same device-resident C5 (and C1) batches; HIP-event times per
launch on one stream; median and min over rounds.  Also checks every variant's output
equals the first's (bit-exact)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    engines = []
    for var in (sys.argv[1:] or ["0", "1024", "2048", "8192"]):
        nbytes, _, smap = var.partition(":")  # seg_bytes[:seg_map]
        os.environ["JRQ_CRC_SEG_BYTES"] = nbytes
        os.environ["JRQ_CRC_SEG_MAP"] = smap or "0"
        e = Engine(0)
        e.use_stream(s.cuda_stream)
        engines.append((f"S{nbytes}/M{smap or 0}", e))
    res = {}
    for cfg, n, eb in (("C5", 64 << 10, 16 << 10), ("C1", 1 << 20, 256)):
        b = W.entry_batch(n, eb, seed=3)
        d = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
             for k, v in b.items() if isinstance(v, np.ndarray)}
        outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in engines]
        times = {name: [] for name, _ in engines}
        for rnd in range(12):
            for (name, e), out in zip(engines, outs):
                a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                e.logentry_checksum_batch_dev(d["etype"], d["index"], d["term"], None,
                                              d["payload"], d["offsets"], out)
                z.record(s)
                z.synchronize()
                if rnd >= 2:
                    times[name].append(a.elapsed_time(z))
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        pay = n * eb
        res[cfg] = {"bit_exact_across_variants": same}
        for name, t in times.items():
            med = float(np.median(t))
            res[cfg][name] = {"ms_median": med, "ms_min": float(np.min(t)),
                              "payload_GBps": pay / (med * 1e-3) / 1e9}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
