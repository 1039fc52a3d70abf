#!/usr/bin/env python3
"""Per-leg kernel durations from rocprofv3 kernel traces, one trace per bench leg
(tools/gpu_check.sh step `legtrace`: `rocprofv3 --kernel-trace -- python bench.py --legs <leg>`,
so every kernel name in a trace carries that leg's workload only), and each leg's roofline
fraction recomputed from them.

For each leg: every kernel name with its launch count and the median / mean / p10 / p90 duration
(us) over all its launches in the pass (warm-up, timed and check launches alike: the median is
the steady state).  With --detail (the bench's full result of a run of the same tree), each
leg's `frac` is recomputed as the leg's algorithmic bytes per launch / the summed medians of its
kernels / 8 TB/s, beside the frac the bench's HIP-event timing gave.

usage: python tools/leg_traces.py gpurun_out [--detail gpurun_out/bench_detail.json] > profiles/<tag>_leg_kernels.json
"""
import csv
import glob
import json
import os
import statistics
import sys

PEAK = 8000.0  # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)

# leg -> (path of its roofline object in the bench detail, kernels of one timed launch)
LEG_KERNELS = {
    "quorum": (("roofline",), ["quorum_epoch_pair_kernel<5, false>"]),
    "table": (("resident_table", "roofline"), ["table_epoch_kernel<5>"]),
    "C2": (("C2", "batched_epochs", "roofline"), ["quorum_epochs_kernel<3,"]),
    "C2L": (("C2", "batched_epochs_64", "roofline"), ["quorum_epochs_kernel<3,"]),
    "C3K": (("C3_k_epochs", "roofline"), ["quorum_epochs_kernel<5,"]),
    "C5": (("crc64", "roofline"), ["crc64_fixed_kernel<true, false>"]),
    "C1": (("C1", "roofline"), ["crc64_fixed_kernel<true, false>"]),
    "ae": (("next_rows", "append_entries_verify", "roofline"),
           ["ae_block_sums", "ae_scan_sums", "ae_meta", "crc64_rounds_kernel<512u, false>",
            "crc64_finish_kernel<true>", "ae_first_corrupt"]),
    "v2": (("next_rows", "v2_decode_verify", "roofline"),
           ["v2_parse", "crc64_fixed_kernel<true, true>", "crc64_rounds_kernel<768u, true>",
            "crc64_finish_kernel<true>", "v2_finish"]),
    "snapshot": (("next_rows", "snapshot_stream_crc64", "roofline"),
                 ["crc64_rounds_kernel<512u, false>", "crc64_finish_kernel<false>"]),
    "lease": (("next_rows", "lease_check", "roofline"), ["lease_check_kernel<5>"]),
    "fanout": (("next_rows", "commit_fanout", "roofline"), ["fanout_eval"]),
}


def kernel_stats(trace_dir):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return None
    durs = {}
    for r in csv.DictReader(open(files[0])):
        name = r["Kernel_Name"]
        durs.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for name, d in sorted(durs.items()):
        d.sort()
        out[name] = {"launches": len(d), "median_us": round(statistics.median(d), 3),
                     "mean_us": round(statistics.fmean(d), 3),
                     "p10_us": round(d[len(d) // 10], 3), "p90_us": round(d[(9 * len(d)) // 10], 3)}
    return out


def main():
    root = sys.argv[1]
    detail = None
    if "--detail" in sys.argv:
        with open(sys.argv[sys.argv.index("--detail") + 1]) as fh:
            detail = json.load(fh)
    res = {"how": __doc__.split("\n\n")[1].replace("\n", " "), "legs": {}}
    for d in sorted(glob.glob(os.path.join(root, "legtrace_*"))):
        leg = os.path.basename(d)[len("legtrace_"):]
        ks = kernel_stats(d)
        if ks is None:
            continue
        entry = {"kernels": ks}
        if leg in LEG_KERNELS:
            path, names = LEG_KERNELS[leg]
            med = 0.0
            found = []
            for n in names:
                hit = [v for k, v in ks.items() if n in k]
                if hit:
                    med += hit[0]["median_us"]
                    found.append(n)
            entry["timed_kernels"] = found
            entry["timed_median_us"] = round(med, 3)
            if detail is not None:
                rl = detail
                for p in path:
                    rl = (rl or {}).get(p)
                if rl and med > 0:
                    frac = rl["bytes_per_launch"] / (med * 1e-6) / 1e9 / PEAK
                    entry["bytes_per_launch"] = rl["bytes_per_launch"]
                    entry["frac_from_trace"] = round(frac, 4)
                    entry["frac_bench_events"] = round(rl["frac"], 4)
                    entry["trace_over_events"] = round(frac / rl["frac"], 4)
        res["legs"][leg] = entry
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
