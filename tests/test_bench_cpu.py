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


def test_launch_cmd_is_one_rank_per_gpu():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_cmd(["--gpus", "8", "--steps", "5"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_world_check():
    sys.path.insert(0, ROOT)
    import bench

    class A:
        gpus, backend = 2, "nccl"
    assert bench.world_check(A, 2, 8) is None
    assert "WORLD_SIZE" in bench.world_check(A, 1, 8)
    assert "visible" in bench.world_check(A, 2, 1)
    A.backend = "gloo"  # a rehearsal may put both ranks on one GPU
    assert bench.world_check(A, 2, 1) is None


def _bench(env_extra, *argv):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                          timeout=300, env=env, cwd=ROOT)


def test_mismatched_world_exits_nonzero():
    p = _bench({"WORLD_SIZE": "1"}, "--gpus", "2")
    assert p.returncode == 2, (p.returncode, p.stderr)
    assert "WORLD_SIZE 1 but --gpus 2" in p.stderr and not p.stdout.strip()


def test_too_few_gpus_exits_nonzero():
    # no WORLD_SIZE: the launcher counts the GPUs in a child first (none here)
    p = _bench({}, "--gpus", "2")
    assert p.returncode == 2, (p.returncode, p.stderr)
    assert "GPU(s) visible" in p.stderr and not p.stdout.strip()
