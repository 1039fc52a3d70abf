#!/usr/bin/env python3
"""Condense rocprofv3 outputs under gpurun_out/ into committed summaries under profiles/.

  python tools/summarize_profiles.py <tag>        (e.g. r02a)

Reads (when present):
  gpurun_out/prof/run_kernel_stats.csv                  rocprofv3 --kernel-trace --stats
  gpurun_out/pmc_<leg>_<COUNTER>/*counter_collection.csv  tools/gpu_check.sh `pmc`: one
      rocprofv3 --pmc pass per bench leg (`bench.py --legs <leg>`) and counter
Writes profiles/<tag>_kernel_stats.csv (verbatim copy) and profiles/<tag>_pmc.json: per leg
and kernel, the mean of each counter over its dispatches, and the HBM bytes per launch
(2 * FETCH_SIZE + WRITE_SIZE) KiB -- on gfx950 FETCH_SIZE counts a wide (16 B per lane)
streaming read at half its bytes (MI355X_MICROARCH.md, HBM section); every product kernel reads
its streams with 16-B loads (the CRC kernels' buffer_load_b128 included), so one rule holds for
all of them (round 2 scaled the CRC kernels by a factor calibrated on one of them, which does
not transfer: VERDICT r02).  `csrc_sha` = bench.csrc_sha() of the tree the passes ran on;
bench.py cites a summary only when it matches its own sources.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
sys.path.insert(0, ROOT)


def kernel_key(name):
    return name.split("(")[0].replace("void ", "")


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[kernel_key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    import bench
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    os.makedirs(PROF, exist_ok=True)
    res = {"tag": tag, "csrc_sha": bench.csrc_sha(), "correction": "2*FETCH_SIZE+WRITE_SIZE (MI355X_MICROARCH.md HBM section), KiB->B; "
           "read_bytes_by_request_size = 32 n32 + 64 n64 + 128 n128 (TCC_EA0_RDREQ_{32,64,128}B) where collected",
           "kernel_stats": {}, "legs": collections.defaultdict(lambda: collections.defaultdict(dict))}
    st = os.path.join(OUT, "prof", "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(st)):
            res["kernel_stats"][kernel_key(r["Name"])] = {"avg_duration_ns": float(r["AverageNs"]),
                                                          "calls": int(r["Calls"])}
    for f in sorted(glob.glob(os.path.join(OUT, "pmc_*_*", "*counter_collection.csv"))):
        d = os.path.basename(os.path.dirname(f))[4:]   # <leg>_<COUNTER>
        leg, counter = d.split("_", 1)
        for k, vals in counters(f).items():
            if "jrq" not in k:
                continue
            for c, v in vals.items():
                res["legs"][leg][k][c] = v
    # per-leg kernel durations from the same passes' kernel traces (one workload per kernel name
    # per pass, unlike the full-bench kernel stats where e.g. C1 and C5 share a kernel name)
    for f in sorted(glob.glob(os.path.join(OUT, "pmc_*_FETCH_SIZE", "*kernel_trace.csv"))):
        leg = os.path.basename(os.path.dirname(f))[4:].rsplit("_FETCH_SIZE", 1)[0]
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if "jrq" in k:
                durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in durs.items():
            v.sort()
            res["legs"][leg][k]["duration_ns_median"] = float(v[len(v) // 2])
            res["legs"][leg][k]["dispatches"] = len(v)
    sizes = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
    for leg, ks in res["legs"].items():
        for k, v in ks.items():
            if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                v["hbm_bytes_per_launch"] = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
                v["hbm_bytes_per_launch_raw"] = (v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
            # the `rdreq` passes: read requests by size, so read bytes need no width rule
            if all(c in v for c in sizes):
                v["read_bytes_by_request_size"] = (32 * v[sizes[0]] + 64 * v[sizes[1]] +
                                                   128 * v[sizes[2]])
                if "WRITE_SIZE" in v:
                    v["hbm_bytes_per_launch_by_request_size"] = (v["read_bytes_by_request_size"] +
                                                                 v["WRITE_SIZE"] * 1024)
    res["legs"] = {k: dict(v) for k, v in res["legs"].items()}
    with open(os.path.join(PROF, f"{tag}_pmc.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True)[:3000])


if __name__ == "__main__":
    main()
