#!/usr/bin/env python3
"""Minimal driver for profiling: a few LogEntry-checksum launches on C5 (or C1) and a few
quorum epochs on C3, device-resident, nothing else in the process."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    e = Engine(0)
    e.use_stream(s.cuda_stream)
    if cfg in ("C5", "C1"):
        n, eb = (64 << 10, 16 << 10) if cfg == "C5" else (1 << 20, 256)
        b = W.entry_batch(n, eb, seed=3)
        d = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
             for k, v in b.items() if isinstance(v, np.ndarray)}
        out = torch.empty(n, dtype=torch.int64, device=dev)
        for _ in range(reps):
            e.logentry_checksum_batch_dev(d["etype"], d["index"], d["term"], None, d["payload"],
                                          d["offsets"], out)
    else:
        b = W.quorum_batch(cfg)
        d = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
             for k, v in b.items()}
        G = d["pending_index"].shape[0]
        c = torch.empty(G, dtype=torch.int64, device=dev)
        st = torch.empty(G, dtype=torch.uint8, device=dev)
        for _ in range(reps):
            e.quorum_epoch_dev(d["match"], d["pending_index"], d["last_appended"],
                               d["last_committed"], d["conf"], c, st)
    torch.cuda.synchronize()
    print("done", cfg)


if __name__ == "__main__":
    main()
