set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_treg.py tests/test_route_gpu.py tests/test_write_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_it16.log 2>&1 || { tail -30 gpurun_out/pytest_it16.log; exit 1; }
tail -1 gpurun_out/pytest_it16.log
TAG=treg16 ARGS="--type treg --steps 10 --warmup 3" FIELDS="kernel_ms_avg frac ms_per_step verified_sampled_keys" bash scripts/ab.sh head new || exit 1
TAG=tlog16 ARGS="--type tlog --steps 8 --warmup 2" FIELDS="converge_ms_avg frac ms_per_step verified_sampled_keys" REPS=1 bash scripts/ab.sh head new || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_it16 -o run --output-format csv -- python3 bench.py --type treg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_treg_it16.log 2>&1 || exit 1
grep -h '^{' gpurun_out/prof_treg_it16.log | cut -c1-150
