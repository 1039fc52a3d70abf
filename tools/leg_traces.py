#!/usr/bin/env python3
"""Per-leg kernel durations from rocprofv3 kernel traces, one trace per bench leg
(tools/gpu_check.sh step `legtrace`: `rocprofv3 --kernel-trace -- python bench.py --legs <leg>`,
so every kernel name in a trace carries that leg's workload only), and each leg's roofline
fraction recomputed from them.

For each leg: every kernel name with its launch count and the median / mean / p10 / p90 duration
(us) over all its launches in the pass; and the timed series of the leg's roofline (the
launches between the bench's start and end marks, `bench.py mark`): its kernels, the kernel time per
launch (summed medians) and the span per launch (first start to last end / launches: what the
bench's event pair measures).  With --detail (the bench's full result of a run of the same
tree), each leg's fraction is recomputed from both, beside the frac the bench's HIP-event
timing gave.

With --trace DIR (one kernel trace of a whole bench run, `rocprofv3 --kernel-trace -- python
bench.py --detail D`) and --detail D of that same run, the run's timed series are matched to
their legs through the result's `timed_series_legs` (the leg of each start mark, in order), so
the recomputed fractions and the bench's come from the same launches.

With --untraced U (the full result of a run of the same tree on the same box without the
tracer, as the driver runs the bench), each leg also gets that run's fraction beside the
trace's: the tracer stretches back-to-back series of short kernels (its per-dispatch completion
signals), so the traced run's own events under-read those legs while its kernel durations do not.
--from-json J re-reads an earlier output instead of a trace (to add --untraced to it).

usage: python tools/leg_traces.py gpurun_out [--detail gpurun_out/bench_detail.json] > profiles/<tag>_leg_kernels.json
       python tools/leg_traces.py --trace gpurun_out/full --detail gpurun_out/full_detail.json [--untraced U]
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
    "quorum": (("roofline",), ["quorum_epoch_pair_kernel<5, false, true>"]),
    "table": (("resident_table", "roofline"), ["table_epoch_kernel<5, false>"]),
    "table_fanout": (("resident_table", "fused_fanout", "roofline"), ["table_epoch_kernel<5, true>"]),
    "C2": (("C2", "batched_epochs", "roofline"), ["quorum_epochs_kernel<3,"]),
    "C2L": (("C2", "batched_epochs_64", "roofline"), ["quorum_epochs_kernel<3,"]),
    "C3K": (("C3_k_epochs", "roofline"), ["quorum_epochs_pair_kernel<5, false, true>"]),
    "C5": (("crc64", "roofline"), ["crc64_fixed_kernel<true, false, 512>"]),
    "C1": (("C1", "roofline"), ["crc64_fixed_kernel<true, false, 1024>"]),
    "ae": (("next_rows", "append_entries_verify", "roofline"),
           ["ae_block_sums", "ae_scan_sums", "ae_meta", "crc64_rounds_kernel<512u, false>",
            "crc64_finish_kernel<true>", "ae_first_corrupt"]),
    "v2": (("next_rows", "v2_decode_verify", "roofline"),
           ["v2_parse", "crc64_fixed_kernel<true, true, 512>", "crc64_rounds_kernel<768u, true>",
            "v2_finish"]),
    "snapshot": (("next_rows", "snapshot_stream_crc64", "roofline"),
                 ["crc64_rounds_kernel<512u, false>", "crc64_finish_kernel<false>"]),
    "lease": (("next_rows", "lease_check", "roofline"), ["leader_tick_pair_kernel<5, false>"]),
    "tick": (("next_rows", "leader_tick", "roofline"), ["leader_tick_pair_kernel<5, true>"]),
    "readindex": (("next_rows", "readindex_quorum", "roofline"), ["readindex_quorum_kernel<5, true>"]),
    "fanout": (("next_rows", "commit_fanout", "roofline"), ["fanout_pair"]),
}


def read_trace(trace_dir):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return None
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(files[0]))]
    rows.sort()
    return rows


def stats(durs):
    d = sorted(durs)
    return {"launches": len(d), "median_us": round(statistics.median(d), 3),
            "mean_us": round(statistics.fmean(d), 3),
            "p10_us": round(d[len(d) // 10], 3), "p90_us": round(d[(9 * len(d)) // 10], 3)}


def is_mark(name):
    return "bitwise_not_kernel" in name or "neg_kernel" in name


def timed_series(rows):
    """The launches between a start mark and the next end mark (bench.py `mark`: a one-element
    bitwise-not right before each timed series' event pair, a negation right after it), as
    lists of (start, end, name)."""
    out, cur = [], None
    for r in rows:
        if "bitwise_not_kernel" in r[2]:
            cur = []
        elif "neg_kernel" in r[2]:
            if cur:
                out.append(cur)
            cur = None
        elif cur is not None:
            cur.append(r)
    return out


def traces(argv, detail):
    """(leg, rows of its launches, its timed series) per leg: one trace per leg (legtrace_<leg>
    directories), or one trace of a whole run split by the run's `timed_series_legs`."""
    if "--trace" in argv:
        rows = read_trace(argv[argv.index("--trace") + 1])
        labels = (detail or {}).get("timed_series_legs")
        series = timed_series(rows)
        if labels is None or len(labels) != len(series):
            raise SystemExit(f"--trace needs the same run's --detail: {len(series)} series in the "
                             f"trace, {None if labels is None else len(labels)} labels")
        for leg in dict.fromkeys(labels):
            ser = [x for x, l in zip(series, labels) if l == leg]
            yield leg, [r for x in ser for r in x], ser
        return
    for d in sorted(glob.glob(os.path.join(argv[1], "legtrace_*"))):
        rows = read_trace(d)
        if rows is not None:
            yield os.path.basename(d)[len("legtrace_"):], rows, timed_series(rows)


def add_untraced(res, plain):
    """Each leg's roofline fraction from an untraced run's full result, beside the trace's."""
    res["untraced_run"] = "frac_untraced_events: the same tree's bench without the tracer, same box"
    for leg, entry in res["legs"].items():
        if leg not in LEG_KERNELS or "frac_from_trace_kernels" not in entry:
            continue
        rl = plain
        for p in LEG_KERNELS[leg][0]:
            rl = (rl or {}).get(p)
        if rl:
            entry["frac_untraced_events"] = round(rl["frac"], 4)
            entry["trace_kernels_over_untraced"] = round(entry["frac_from_trace_kernels"] / rl["frac"], 4)


def main():
    if "--from-json" in sys.argv:
        with open(sys.argv[sys.argv.index("--from-json") + 1]) as fh:
            res = json.load(fh)
        with open(sys.argv[sys.argv.index("--untraced") + 1]) as fh:
            add_untraced(res, json.load(fh))
        json.dump(res, sys.stdout, indent=1)
        print()
        return
    detail = None
    if "--detail" in sys.argv:
        with open(sys.argv[sys.argv.index("--detail") + 1]) as fh:
            detail = json.load(fh)
    res = {"how": "\n\n".join(__doc__.split("\n\n")[1:3]).replace("\n", " "), "legs": {}}
    if "--trace" in sys.argv:
        res["trace"] = "one trace of the whole run (the launches of the leg's timed series only)"
    for leg, rows, series in traces(sys.argv, detail):
        durs = {}
        for a, b, n in rows:
            if not is_mark(n):
                durs.setdefault(n, []).append((b - a) / 1e3)
        entry = {"kernels": {n: stats(v) for n, v in sorted(durs.items())}}
        if leg in LEG_KERNELS:
            path, names = LEG_KERNELS[leg]
            # the timed series of this leg's roofline: the first series holding every kernel of
            # one timed launch and the fewest other names
            best = None
            for ser in series:
                kn = {n for _, _, n in ser}
                if all(any(x in k for k in kn) for x in names):
                    if best is None or len(kn) < len({n for _, _, n in best}):
                        best = ser
            if best is not None:
                main = [n for _, _, n in best if names[0] in n]
                launches = len(main)
                per = {}
                for a, b, n in best:
                    per.setdefault(n, []).append((b - a) / 1e3)
                kern = sum(statistics.median(v) * len(v) / launches for v in per.values())
                span = (best[-1][1] - best[0][0]) / 1e3 / launches
                entry["timed_series"] = {"launches": launches,
                                         "kernels": {n: stats(v) for n, v in sorted(per.items())},
                                         "kernel_us_per_launch": round(kern, 3),
                                         "span_us_per_launch": round(span, 3)}
                if detail is not None:
                    rl = detail
                    for p in path:
                        rl = (rl or {}).get(p)
                    if rl:
                        B = rl["bytes_per_launch"]
                        entry["bytes_per_launch"] = B
                        entry["frac_from_trace_kernels"] = round(B / (kern * 1e-6) / 1e9 / PEAK, 4)
                        entry["frac_from_trace_span"] = round(B / (span * 1e-6) / 1e9 / PEAK, 4)
                        entry["frac_bench_events"] = round(rl["frac"], 4)
                        entry["span_over_events"] = round(entry["frac_from_trace_span"] / rl["frac"], 4)
        res["legs"][leg] = entry
    if "--untraced" in sys.argv:
        with open(sys.argv[sys.argv.index("--untraced") + 1]) as fh:
            add_untraced(res, json.load(fh))
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
