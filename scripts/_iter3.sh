set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in cnt; do
JY_LIB=$PWD/jylis_amd/_ab/libjylis_$L.so timeout -k 10 300 python -u -m pytest tests/test_route_gpu.py tests/test_route_dist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_it3_$L.log 2>&1 || { tail -30 gpurun_out/pytest_it3_$L.log; exit 1; }
tail -1 gpurun_out/pytest_it3_$L.log
done
JY_TRACE=1 timeout -k 10 300 python bench.py --type e2e --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_e2e_it3.log 2>&1 || { tail -20 gpurun_out/bench_e2e_it3.log; exit 1; }
grep -h '^{' gpurun_out/bench_e2e_it3.log | cut -c1-700
TAG=treg3 ARGS="--type treg --route --steps 10 --warmup 3" FIELDS="step_ms_avg_events verified_sampled_keys" bash scripts/ab.sh head cnt cntp cntr new || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_uj_it3 -o run --output-format csv -- python3 bench.py --type ujson --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_uj_it3.log 2>&1 || exit 1
echo done
