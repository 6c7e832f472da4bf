set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
JY_LIB=$PWD/jylis_amd/_ab/libjylis_nofence.so timeout -k 10 300 python -u -m pytest tests/test_host_copy_gpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_it7_nofence.log 2>&1; echo "nofence rc=$?"; tail -3 gpurun_out/pytest_it7_nofence.log
timeout -k 10 300 python -u -m pytest tests/test_host_copy_gpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_it7.log 2>&1; echo "fence rc=$?"; tail -3 gpurun_out/pytest_it7.log
JY_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_uj_it7 -o run --output-format csv -- python3 bench.py --type ujson --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_uj_it7.log 2>&1 || exit 1
grep -h '^{' gpurun_out/prof_uj_it7.log | cut -c1-200
