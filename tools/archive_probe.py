#!/usr/bin/env python3
"""Probe: 1 GiB as one snapshot-archive stream vs 64k region streams (jrq_crc64_stream_update_dev),
HIP-event timing per leg; run under rocprofv3 --kernel-trace --stats to split the kernels.
  python tools/archive_probe.py [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sofa-jraft_amd"))


def main():
    import torch

    from jraft_amd import Engine
    from jraft_amd import workloads as W
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    e = Engine(0)
    e.use_stream(s.cuda_stream)
    tot = 1 << 30
    pay = torch.from_numpy(W.random_bytes(3, tot)).to(dev)
    legs = {"archive": torch.tensor([0, tot], dtype=torch.int64, device=dev),
            "regions": torch.arange(0, tot + 1, 16 << 10, dtype=torch.int64, device=dev),
            "archive_x16": torch.arange(0, tot + 1, 64 << 20, dtype=torch.int64, device=dev)}
    for name, off in legs.items():
        reg = torch.zeros(off.numel() - 1, dtype=torch.int64, device=dev)
        for _ in range(3):
            e.crc64_stream_update_dev(reg, pay, off)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            e.crc64_stream_update_dev(reg, pay, off)
        b.record(s)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / reps
        print(f"{name:12s} S={off.numel() - 1:6d} {ms * 1e3:8.1f} us  {tot / ms / 1e6:7.1f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
