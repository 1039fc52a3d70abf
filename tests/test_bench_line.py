"""bench.py's printed line stays within what the driver parses (the 20.8 KB line of
round 3 came back `parsed: null`; round 2's 13.2 KB line was parsed).  The line is built from a
real full result (profiles/r03f_bench.json: every leg of the default run) by the same
compact_line / emit_line the bench calls."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
ROOFLINE = ("bound", "achieved", "peak", "unit", "frac", "traffic")


def _full():
    with open(os.path.join(ROOT, "profiles", "r03f_bench.json")) as fh:
        return json.load(fh)


def test_line_under_budget_with_contract_keys(tmp_path):
    full = _full()
    s = bench.emit_line(full, str(tmp_path / "detail.json"))
    assert "\n" not in s
    assert len(s) <= bench.LINE_BUDGET
    line = json.loads(s)
    for k in CONTRACT:
        assert k in line, k
    for k in ROOFLINE:
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["value"] == full["value"] or abs(line["value"] / full["value"] - 1) < 1e-5
    assert line["crc64"]["unit"].startswith("GB/s")
    # every leg of the full run has its summary, each with the four fields the verdict asks for
    for leg in ("quorum_C3", "table", "C2_epochs", "C5_verify", "C1", "append_entries_verify",
                "v2_decode_verify", "snapshot_stream_crc64", "lease_check", "commit_fanout"):
        assert {"ms", "frac", "bit_exact"} <= set(line["legs"][leg]), leg
    # the detail file holds the whole result
    with open(tmp_path / "detail.json") as fh:
        assert json.load(fh) == full


def test_line_budget_with_every_rank_field(tmp_path):
    """An N = 8 line (per-rank CRC rates, multi_gpu) stays within the budget too."""
    full = _full()
    full["n_gpus"] = 8
    full["crc64"]["per_rank_GBps"] = [5402.25567] * 8
    full["crc64"]["per_rank_bit_exact"] = [True] * 8
    full["multi_gpu"]["publish_ms"] = 0.0123456
    s = bench.emit_line(full, str(tmp_path / "d.json"))
    assert len(s) <= bench.LINE_BUDGET
    assert json.loads(s)["crc64"]["per_rank_GBps"][7] > 0
