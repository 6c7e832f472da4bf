set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_it2.log 2>&1 || { tail -30 gpurun_out/pytest_it2.log; exit 1; }
tail -1 gpurun_out/pytest_it2.log
timeout -k 10 300 python bench.py --type e2e --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_e2e_it2.log 2>&1 || { tail -20 gpurun_out/bench_e2e_it2.log; exit 1; }
grep -h '^{' gpurun_out/bench_e2e_it2.log | cut -c1-1200
TAG=tlog ARGS="--type tlog --steps 8 --warmup 2" FIELDS="converge_ms_avg kernel_ms_avg frac verified_sampled_keys" bash scripts/ab.sh new head || exit 1
TAG=treg ARGS="--type treg --route --steps 10 --warmup 3" FIELDS="ms_per_step step_ms_avg_events verified_sampled_keys" bash scripts/ab.sh new head rt1 rt2 ru2 ru2w || exit 1
timeout -k 10 120 python3 - <<'PY'
import torch, time
x = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True); d = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
for _ in range(3): d.copy_(x, non_blocking=True)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(10): d.copy_(x, non_blocking=True)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
print("pinned H2D 64 MiB: %.1f GB/s" % (x.numel() / dt / 1e9))
y = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
t = time.perf_counter()
for _ in range(10): y.copy_(d, non_blocking=True)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
print("pinned D2H 64 MiB: %.1f GB/s" % (x.numel() / dt / 1e9))
PY
