#!/usr/bin/env python3
"""v2_boundary_probe.py -- what the V2 read path's CRC pass would cost with one entry boundary
per record instead of two (tools only; not part of the product).

On the C5-shaped V2 records (64k x 16 KiB data) it times the batched CRC kernels over
  (a) the interleaved list the product hashes: gap, data, gap, ... (2N+1 ranges);
  (b) data starts only: [data_start_i, data_start_{i+1}) (N+1 ranges) -- each range then holds
      one record's data followed by its trailer and the next header, whose CRC could be
      removed by an inverse shift of a few dozen bytes;
  (c) the records themselves (N ranges, the C5-like aligned case for comparison).
with HIP events around 20 back-to-back launches each.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    eng = Engine(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    eng.use_stream(stream.cuda_stream)
    c5 = W.CONFIGS["C5"]
    n = c5["groups"]
    eb = W.entry_batch(n, c5["entry_bytes"], seed=W.SEED_BASE ^ 5)
    rec, roff = W.v2_records(eb["etype"], eb["index"], eb["term"], eb["payload"], eb["offsets"],
                             np.zeros(n, np.uint64))
    d = eng.v2_decode_verify(rec, roff)
    ds, dl = d["data_off"].astype(np.uint64), d["data_len"].astype(np.uint64)
    inter = np.empty(2 * n + 2, np.uint64)
    inter[0] = 0
    inter[1:2 * n + 1:2] = ds
    inter[2:2 * n + 1:2] = ds + dl
    inter[2 * n + 1] = len(rec)
    starts = np.concatenate([[0], ds, [len(rec)]]).astype(np.uint64)
    lists = {"interleaved (2N+1)": inter, "data starts (N+1)": starts,
             "records (N)": roff.astype(np.uint64)}
    d_rec = torch.from_numpy(rec).to(dev)
    for name, offs in lists.items():
        assert (np.diff(offs.astype(np.int64)) >= 0).all()
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        out = torch.empty(len(offs) - 1, dtype=torch.int64, device=dev)
        for _ in range(3):
            eng.crc64_batch_dev(d_rec, d_off, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            eng.crc64_batch_dev(d_rec, d_off, out)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"{name:22s} {len(offs) - 1:7d} ranges  {ms * 1e3:7.1f} us  "
              f"{len(rec) / (ms * 1e-3) / 1e9:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
