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


@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_host_mirror_under_sanitizers(san):
    """The whole list -- concurrent callers with the background flusher, multi-threaded pack
    and deliver, re-entrancy, the differential tests -- under ThreadSanitizer and under
    AddressSanitizer + UBSan, on the CPU: the host mirror linked against the test double of
    libjrq (tests/cpp/fake_jrq.cpp, the oracle's BallotBox replay as the epoch)."""
    b = os.path.join(ROOT, "tests", "_build", "host_test_" + san)
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "san"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([b, "gpu"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-8000:]
    assert "testConcurrentCallersWide" in r.stdout and "0 failed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr


@pytest.mark.gpu
def test_host_mirror_on_gpu():
    out = _run("gpu")
    assert "testManyGroupsJointConsensusOnGpu" in out and "testRandomDifferentialOnGpu" in out
    assert "testConcurrentCallersWide" in out
    assert "0 failed" in out
