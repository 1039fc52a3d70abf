#!/usr/bin/env python3
"""A/B probe: LogEntry checksum GB/s on aligned vs ragged layouts, and the V2 read path.
JRQ_LIB selects the libjrq.so under test.  Prints one line per case."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sofa-jraft_amd"), os.path.join(ROOT, "oracle")]


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    e = Engine(0)
    e.use_stream(s.cuda_stream)
    rng = np.random.default_rng(1)

    def timeit(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    cases = [("C5 aligned 64k x 16KiB", 64 << 10, 16 << 10, 0),
             ("C5 ragged 64k x 16KiB+-", 64 << 10, 16 << 10, 1),
             ("C1 1M x 256B", 1 << 20, 256, 0),
             ("ragged 4M x ~256B", 4 << 20, 256, 1)]
    for name, n, eb, ragged in cases:
        b = W.entry_batch(n, eb, seed=3)
        if ragged:
            lens = rng.integers(eb // 2, eb + eb // 2, n).astype(np.uint64)
            offs = np.zeros(n + 1, np.uint64)
            offs[1:] = np.cumsum(lens)
            b["offsets"] = offs
            b["payload"] = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
        d = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
             for k, v in b.items() if isinstance(v, np.ndarray)}
        out = torch.empty(n, dtype=torch.int64, device=dev)
        ms = timeit(lambda: e.logentry_checksum_batch_dev(d["etype"], d["index"], d["term"], None,
                                                          d["payload"], d["offsets"], out))
        pay = int(b["offsets"][-1] - b["offsets"][0])
        print(f"{name}: {ms * 1e3:.1f} us  {pay / ms / 1e6:.0f} GB/s", flush=True)
        if name.startswith("C5 aligned"):
            ck = out.cpu().numpy().view(np.uint64)
            rec, roff = W.v2_records(b["etype"], b["index"], b["term"], b["payload"], b["offsets"], ck)
            d_rec = torch.from_numpy(rec).to(dev)
            d_roff = torch.from_numpy(roff.view(np.int64)).to(dev)
            o = {k: torch.empty(n, dtype={np.uint8: torch.uint8, np.uint32: torch.int32}.get(t, torch.int64), device=dev)
                 for k, t in Engine.V2_FIELDS}
            ms = timeit(lambda: e.v2_decode_verify_dev(d_rec, d_roff, o))
            ok = bool((o["computed"].cpu().numpy().view(np.uint64) == ck).all())
            print(f"V2 decode 64k x 16KiB: {ms * 1e3:.1f} us  {rec.size / ms / 1e6:.0f} GB/s ok={ok}", flush=True)
        del d, out
    e.close()


if __name__ == "__main__":
    main()
