#!/bin/bash
# TLOG parity tests + bench (+ optional rocprof stats), each step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-tl}
timeout -k 10 600 python -u -m pytest tests/test_parity_tlog.py tests/test_tlog_write_gpu.py tests/test_arena_gpu.py \
  tests/test_route_csr_gpu.py tests/test_docs_converge.py -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python bench.py --type tlog --steps ${STEPS:-8} --warmup 2 --batches 4 --no-cpu-baseline \
  > gpurun_out/bench_tlog_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_tlog_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_tlog_$TAG.log | cut -c1-1500
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlog_$TAG -o run --output-format csv \
    -- python3 bench.py --type tlog --steps ${PSTEPS:-20} --warmup 2 --batches 4 --no-cpu-baseline > gpurun_out/prof_tlog_$TAG.log 2>&1 || exit 1
  python3 scripts/kstats.py gpurun_out/prof_tlog_$TAG/run_kernel_stats.csv 12
fi
