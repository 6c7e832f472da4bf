set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
JY_LIB=$PWD/jylis_amd/_ab/libjylis_nofence.so timeout -k 10 300 python -u -m pytest tests/test_host_copy_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_it6_nofence.log 2>&1; echo "nofence rc=$?"; tail -3 gpurun_out/pytest_it6_nofence.log
timeout -k 10 300 python -u -m pytest tests/test_host_copy_gpu.py tests/test_converge_keys_gpu.py tests/test_keys_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_it6.log 2>&1 || { tail -30 gpurun_out/pytest_it6.log; exit 1; }
tail -1 gpurun_out/pytest_it6.log
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --type ujson --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/uj6_$rep.log 2>&1 || exit 1
  echo "uj $rep $(grep -h '^{' gpurun_out/uj6_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['per_converge']['touched_cloud'], d['roofline']['converge_ms_avg'], d['verified_sampled_docs'])")"
done
timeout -k 10 300 python bench.py --type e2e --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_e2e_it6.log 2>&1 || exit 1
grep -h '^{' gpurun_out/bench_e2e_it6.log | cut -c1-900
