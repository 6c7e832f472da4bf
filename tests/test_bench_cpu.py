"""bench.py host logic that runs without a GPU: the hang watchdog exits
non-zero (a routed collective that hangs is a failure, not a clean line),
and the parallel CPU baseline sizes itself to the CPUs it may really use."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_exits_nonzero():
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.watchdog(0.3, {'metric': 'm', 'value': 1.0}, 0); time.sleep(20); print('not reached')" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 3, (p.returncode, p.stdout, p.stderr)
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert "error" in line["routed"] and line["value"] == 1.0
    assert "not reached" not in p.stdout


def test_watchdog_cancelled_phase_exits_zero():
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "d = bench.watchdog(5.0, {}, 0); d.cancel(); print('done')" % ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == "done"


def test_cpu_share_is_the_usable_set():
    sys.path.insert(0, ROOT)
    import bench
    n, how = bench.cpu_share()
    assert 1 <= n <= (os.cpu_count() or 1)
    if hasattr(os, "sched_getaffinity"):
        assert n <= len(os.sched_getaffinity(0))
    assert "sched_getaffinity" in how or "cpu_count" in how
