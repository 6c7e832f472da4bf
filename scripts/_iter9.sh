set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_tlog.py tests/test_tlog_write_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_it9.log 2>&1 || { tail -30 gpurun_out/pytest_it9.log; exit 1; }
tail -1 gpurun_out/pytest_it9.log
JY_LIB=$PWD/jylis_amd/_ab/libjylis_w7.so timeout -k 10 300 python -u -m pytest tests/test_parity_tlog.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_it9_w7.log 2>&1 || { tail -30 gpurun_out/pytest_it9_w7.log; exit 1; }
tail -1 gpurun_out/pytest_it9_w7.log
TAG=tlog9 ARGS="--type tlog --steps 8 --warmup 2" FIELDS="converge_ms_avg ms_per_step verified_sampled_keys" bash scripts/ab.sh head new w7 w8 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_tlog_it9 -o run --output-format csv -- python3 bench.py --type tlog --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tlog_it9.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_uj_it9 -o run --output-format csv -- python3 bench.py --type ujson --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_uj_it9.log 2>&1 || exit 1
grep -h '^{' gpurun_out/prof_uj_it9.log | cut -c1-200
