#!/usr/bin/env python3
"""Host cost per prepared quorum-epoch launch (tools only): time N launches of a tiny epoch
(64 groups) from Python, the C ABI call, and a bare hipLaunch of torch's for scale."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def main():
    import torch
    from jraft_amd import Engine, workloads as W
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    e = Engine(0)
    e.use_stream(s.cuda_stream)
    b = W.quorum_batch("C3", groups=64)
    d = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev) for k, v in b.items()}
    c = torch.empty(64, dtype=torch.int64, device=dev)
    st = torch.empty(64, dtype=torch.uint8, device=dev)
    f = e.quorum_epoch_launcher(d["match"], d["pending_index"], d["last_appended"], d["last_committed"], d["conf"], c, st)
    x = torch.zeros(64, device=dev)
    for name, fn in (("prepared", f), ("torch add_", lambda: x.add_(1.0)),
                     ("quorum_epoch_dev", lambda: e.quorum_epoch_dev(d["match"], d["pending_index"], d["last_appended"], d["last_committed"], d["conf"], c, st))):
        for _ in range(200):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2000):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{name:18s} host {1e6 * (t1 - t0) / 2000:.2f} us/call")


if __name__ == "__main__":
    main()
