#!/bin/bash
# Counter block-merge change: the counter tests, the headline, GCOUNT and GET
# lines, a kernel trace of the headline and the PMC traffic passes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 600 python -u -m pytest tests/test_parity_counters.py tests/test_docs_converge.py tests/test_node_gpu.py \
  tests/test_write_gpu.py tests/test_converge_keys_gpu.py -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_cnt_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_cnt_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_cnt_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_$TAG.log | cut -c1-200
for m in gcount read; do
  timeout -k 10 400 python bench.py --type $m --steps 8 --warmup 2 > gpurun_out/bench_${m}_$TAG.log 2>&1 || exit 1
  grep -h '^{' gpurun_out/bench_${m}_$TAG.log | cut -c1-200
done
TAG=$TAG bash scripts/gpu_profile.sh
