#!/bin/bash
# Routed TREG after a partition / receiver change: the routing tests, the
# plain and routed bench lines and a kernel trace of the routed one.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 600 python -u -m pytest tests/test_route_gpu.py tests/test_route_dist_gpu.py tests/test_parity_treg.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_route_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_route_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_route_$TAG.log
for v in "" "--route"; do
  n=$(echo "$v" | tr -d ' -')
  timeout -k 10 400 python bench.py --type treg $v --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_treg${n}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_treg${n}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_treg${n}_$TAG.log | cut -c1-400
done
bash scripts/gpu_treg_route_prof.sh
