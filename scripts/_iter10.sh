set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 400 python -u -m pytest tests/test_stage_determinism_gpu.py -x -q --timeout 380 --timeout-method thread > gpurun_out/pytest_it10_$rep.log 2>&1; echo "det $rep rc=$?"; tail -3 gpurun_out/pytest_it10_$rep.log
done
for rep in 1 2 3; do
for v in head new; do
  L=$PWD/jylis_amd/libjylis_gpu.so; [ $v = head ] && L=$PWD/jylis_amd/_ab/libjylis_head.so
  JY_LIB=$L timeout -k 10 300 python3 bench.py --type ujson --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/uj10_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/uj10_${v}_$rep.log; exit 1; }
  echo "$v $rep $(grep -h '^{' gpurun_out/uj10_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['per_converge']['touched_cloud'], d['roofline']['converge_ms_avg'], d['verified_sampled_docs'])")"
done
done
timeout -k 10 300 python -u -m pytest tests/test_parity_tlog.py tests/test_tlog_write_gpu.py tests/test_docs_converge.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_it10_tlog.log 2>&1 || { tail -30 gpurun_out/pytest_it10_tlog.log; exit 1; }
tail -1 gpurun_out/pytest_it10_tlog.log
TAG=tlog10 ARGS="--type tlog --steps 8 --warmup 2" FIELDS="converge_ms_avg ms_per_step verified_sampled_keys" bash scripts/ab.sh head new || exit 1
