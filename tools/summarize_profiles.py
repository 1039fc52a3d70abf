#!/usr/bin/env python3
"""Condense rocprofv3 outputs under gpurun_out/ into committed summaries under profiles/.

  python tools/summarize_profiles.py <tag>        (e.g. r01)

Reads (when present):
  gpurun_out/prof/run_kernel_stats.csv            rocprofv3 --kernel-trace --stats
  gpurun_out/pmc_fetch/run_counter_collection.csv rocprofv3 --kernel-trace --pmc FETCH_SIZE
  gpurun_out/pmc_write/run_counter_collection.csv rocprofv3 --kernel-trace --pmc WRITE_SIZE
  gpurun_out/pmc*_C*/run_counter_collection.csv   tools/pmc_crc.sh SQ / TCC groups
Writes profiles/<tag>_kernel_stats.csv (verbatim copy) and profiles/<tag>_pmc.json:
per kernel, the mean of each counter over its dispatches.  HBM traffic per launch is
(2 * FETCH_SIZE + WRITE_SIZE) KiB: on gfx950 FETCH_SIZE counts 128-B read requests as
64 B, i.e. half the bytes of a wide streaming read (MI355X_MICROARCH.md, HBM section);
the raw values are kept next to the corrected ones.
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


def kernel_key(name):
    return name.split("(")[0].replace("void ", "")


def counters(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[kernel_key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(PROF, exist_ok=True)
    res = {"tag": tag, "kernels": collections.defaultdict(dict)}
    st = os.path.join(OUT, "prof", "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(st)):
            res["kernels"][kernel_key(r["Name"])]["avg_duration_ns"] = float(r["AverageNs"])
            res["kernels"][kernel_key(r["Name"])]["calls"] = int(r["Calls"])
    files = glob.glob(os.path.join(OUT, "pmc_*", "*counter_collection.csv")) + \
        glob.glob(os.path.join(OUT, "pmc*_C*", "*counter_collection.csv"))
    for f in sorted(files):
        src = os.path.basename(os.path.dirname(f))
        for k, d in counters(f).items():
            for c, v in d.items():
                res["kernels"][k][c] = v
                res["kernels"][k].setdefault("sources", []).append(f"{src}:{c}")
    for k, d in res["kernels"].items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch_corrected"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
            d["hbm_bytes_per_launch_raw"] = (d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    res["kernels"] = {k: v for k, v in res["kernels"].items() if "jrq" in k}
    with open(os.path.join(PROF, f"{tag}_pmc.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True)[:4000])


if __name__ == "__main__":
    main()
