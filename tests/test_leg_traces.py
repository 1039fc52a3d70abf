"""tools/leg_traces.py on a synthetic whole-run trace: timed series are matched to their legs by
the run's `timed_series_legs`, and each leg's fraction is recomputed from its own launches only
(two legs here run the same kernel template, as C5 and C1 do)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_trace(d, rows):
    os.makedirs(d)
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for name, a, b in rows:
            w.writerow([name, a, b])


def test_whole_run_trace_split_by_labels(tmp_path):
    fixed = "void jrq::crc64_fixed_kernel<true, false, 512>(JrqCrcArgs)"
    wide = "void jrq::crc64_fixed_kernel<true, false, 1024>(JrqCrcArgs)"
    rows, t = [], 0

    def series(name, dur_ns, n):
        nonlocal t
        rows.append(("void at::native::bitwise_not_kernel(...)", t, t + 1000))
        t += 2000
        for _ in range(n):
            rows.append((name, t, t + dur_ns))
            t += dur_ns
        rows.append(("void at::native::neg_kernel(...)", t, t + 1000))
        t += 5000

    series(fixed, 175_000, 4)   # C5: 1 GB per launch
    series("other_kernel", 10_000, 3)  # an unlabelled leg's series
    series(wide, 60_000, 4)     # C1: the same kernel's one-lane-per-entry form, 0.3 GB per launch
    trace = tmp_path / "full"
    _write_trace(str(trace), rows)
    detail = {"timed_series_legs": ["C5", "drive", "C1"],
              "crc64": {"roofline": {"bytes_per_launch": 1_000_000_000, "frac": 0.7}},
              "C1": {"roofline": {"bytes_per_launch": 300_000_000, "frac": 0.6}}}
    dp = tmp_path / "detail.json"
    dp.write_text(json.dumps(detail))
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "tools", "leg_traces.py"),
                                   "--trace", str(trace), "--detail", str(dp)])
    legs = json.loads(out)["legs"]
    assert legs["C5"]["timed_series"]["launches"] == 4
    assert legs["C5"]["timed_series"]["kernel_us_per_launch"] == 175.0
    assert abs(legs["C5"]["frac_from_trace_kernels"] - 1e9 / 175e-6 / 1e9 / 8000) < 1e-4
    assert legs["C1"]["timed_series"]["kernel_us_per_launch"] == 60.0
    assert abs(legs["C1"]["frac_from_trace_kernels"] - 0.3e9 / 60e-6 / 1e9 / 8000) < 1e-4
    assert "timed_series" not in legs["drive"]


def test_whole_run_trace_needs_matching_labels(tmp_path):
    trace = tmp_path / "full"
    _write_trace(str(trace), [("void at::native::bitwise_not_kernel(...)", 0, 1),
                              ("k", 2, 3), ("void at::native::neg_kernel(...)", 4, 5)])
    dp = tmp_path / "detail.json"
    dp.write_text(json.dumps({"timed_series_legs": ["C5", "C1"]}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "leg_traces.py"),
                        "--trace", str(trace), "--detail", str(dp)], capture_output=True, text=True)
    assert r.returncode != 0 and "1 series in the trace, 2 labels" in r.stderr
