set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_route_csr_gpu.py tests/test_route_dist_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_route2.log 2>&1 || { tail -30 gpurun_out/pytest_route2.log; exit 1; }
tail -2 gpurun_out/pytest_route2.log
for m in tlog ujson; do
  timeout -k 10 400 python bench.py --type $m --route --steps 6 --warmup 2 --batches 3 --no-cpu-baseline > gpurun_out/bench_${m}_route.log 2>&1 || { tail -20 gpurun_out/bench_${m}_route.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${m}_route.log | cut -c1-900
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --type tlog --backend gloo --keys 1000000 --steps 4 --warmup 1 --batches 2 --no-cpu-baseline > gpurun_out/bench_tlog_gloo2.log 2>&1 || { tail -20 gpurun_out/bench_tlog_gloo2.log; exit 1; }
grep -h '^{' gpurun_out/bench_tlog_gloo2.log | cut -c1-900
