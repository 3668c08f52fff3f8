"""bench.py's C4 watchdog (run_guarded) with a stub leg, on CPU.

The C4 leg replaces the reference's mp.Queue hand-off (/root/reference/SLAM.py:13,18-23) with a
shared host batch + RCCL gather; a collective that never completes must end the rank non-zero,
with the main JSON line printed and the shared-memory segment unlinked."""
import json
import os
import subprocess
import sys

from conftest import ROOT

STUB = r"""
import sys, time
sys.path.insert(0, %r)
import bench
from multiprocessing import shared_memory

def leg(segments):
    shm = shared_memory.SharedMemory(name=%r, create=True, size=1 << 16)
    segments.append(shm)
    %s

res = bench.run_guarded(leg, %r, 0, {"metric": "m", "value": 1.0})
print("RETURNED", res)
"""


def _run(name, body, timeout):
    code = STUB % (ROOT, name, body, timeout)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)


def test_timeout_exits_nonzero_prints_line_and_unlinks():
    name = "lslam_wdtest_%d" % os.getpid()
    p = _run(name, "time.sleep(30)", 1.0)
    try:
        assert p.returncode == 3, (p.returncode, p.stderr)
        line = json.loads(p.stdout.strip().splitlines()[-1])
        assert line["value"] == 1.0 and line["c4"]["error"].startswith("timeout")
        assert "RETURNED" not in p.stdout
        assert not os.path.exists("/dev/shm/" + name), "segment leaked"
        assert "leaked shared_memory" not in p.stderr
    finally:
        if os.path.exists("/dev/shm/" + name):
            os.unlink("/dev/shm/" + name)


def test_leg_error_is_reported_not_fatal():
    name = "lslam_wdtest_e%d" % os.getpid()
    p = _run(name, "shm.close(); shm.unlink(); raise RuntimeError('boom')", 30.0)
    assert p.returncode == 0, p.stderr
    assert "RETURNED {'error': 'RuntimeError: boom'}" in p.stdout
    assert not os.path.exists("/dev/shm/" + name)


def test_leg_result_passes_through():
    name = "lslam_wdtest_o%d" % os.getpid()
    p = _run(name, "shm.close(); shm.unlink(); return {'ok': 1}", 30.0)
    assert p.returncode == 0, p.stderr
    assert "RETURNED {'ok': 1}" in p.stdout
