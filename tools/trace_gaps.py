"""Per-kernel durations and the gaps between consecutive kernels of one stream, from a
rocprofv3 --kernel-trace CSV (tools/gpu_check.sh step `trace`): where an op's wall time goes
besides its kernels (launch gaps, no-op launches).

usage: python tools/trace_gaps.py gpurun_out/trace_v2 [--last N]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 40
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    by_q = defaultdict(list)
    for r in rows:
        by_q[r.get("Queue_Id", "0")].append(r)
    for q, rs in by_q.items():
        print(f"queue {q}: {len(rs)} dispatches; the last {last}:")
        prev_end = None
        for r in rs[-last:]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            print(f"  {r['Kernel_Name'][:60]:60s} dur {(e - s) / 1e3:8.2f} us  gap {gap:7.2f} us")
            prev_end = e


if __name__ == "__main__":
    main()
