#!/bin/bash
# TREG after a kernel / fold change: the TREG-touching tests, the plain and
# routed bench lines, and a kernel trace of the plain line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 600 python -u -m pytest tests/test_parity_treg.py tests/test_route_gpu.py tests/test_write_gpu.py \
  tests/test_arena_gpu.py tests/test_node_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_treg_$TAG.log 2>&1 \
  || { tail -30 gpurun_out/pytest_treg_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_treg_$TAG.log
for v in "" "--route"; do
  n=$(echo "$v" | tr -d ' -')
  timeout -k 10 400 python bench.py --type treg $v --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_treg${n}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_treg${n}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_treg${n}_$TAG.log | cut -c1-700
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_$TAG -o run --output-format csv \
  -- python3 bench.py --type treg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_treg_$TAG.log 2>&1 || exit 1
echo "treg quick done"
