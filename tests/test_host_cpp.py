"""Runs the C++ host-mirror tests (tests/cpp/host_test.cpp): BallotBoxTest / BallotTest /
LogEntryTest / CrcUtilTest re-expressed against jraft::BallotBox, LogEntry, CrcUtil."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_build", "host_test")


def _run(mode):
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    r = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_host_mirror_cpu_semantics():
    out = _run("cpu")
    assert "0 failed" in out


@pytest.mark.gpu
def test_host_mirror_on_gpu():
    out = _run("gpu")
    assert "testManyGroupsJointConsensusOnGpu" in out and "testRandomDifferentialOnGpu" in out
    assert "0 failed" in out
