set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-it}
timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py tests/test_route_dist_gpu.py tests/test_keys_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -1 gpurun_out/pytest_$T.log
timeout -k 10 300 python bench.py --type e2e --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_e2e_$T.log 2>&1 || { tail -20 gpurun_out/bench_e2e_$T.log; exit 1; }
grep -h '^{' gpurun_out/bench_e2e_$T.log | cut -c1-900
timeout -k 10 300 python bench.py --type treg --route --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_treg_route_$T.log 2>&1 || exit 1
grep -h '^{' gpurun_out/bench_treg_route_$T.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_route_$T -o run --output-format csv -- python3 bench.py --type treg --route --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_treg_route_$T.log 2>&1 || exit 1
python scripts/kstats.py gpurun_out/prof_treg_route_$T/run_kernel_stats.csv | head -12
