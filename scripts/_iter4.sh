set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py tests/test_route_dist_gpu.py tests/test_converge_keys_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_it4.log 2>&1 || { tail -30 gpurun_out/pytest_it4.log; exit 1; }
tail -1 gpurun_out/pytest_it4.log
JY_TRACE=1 timeout -k 10 300 python bench.py --type e2e --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_e2e_it4.log 2>&1 || { tail -20 gpurun_out/bench_e2e_it4.log; exit 1; }
grep -h '^{' gpurun_out/bench_e2e_it4.log | cut -c1-300
TAG=treg4 ARGS="--type treg --route --steps 10 --warmup 3" FIELDS="step_ms_avg_events verified_sampled_keys" bash scripts/ab.sh head new || exit 1

TAG=uj4 ARGS="--type ujson --steps 16 --warmup 2" FIELDS="converge_ms_avg frac verified_sampled_docs" bash scripts/ab.sh head new || exit 1
echo done2
