#!/bin/bash
# TLOG after a kernel change: the TLOG tests, the bench line (twice) and a
# kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 600 python -u -m pytest tests/test_parity_tlog.py tests/test_write_gpu.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_tlog_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_tlog_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_tlog_$TAG.log
for r in 1 2; do
  timeout -k 10 400 python bench.py --type tlog --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_tlog${r}_$TAG.log 2>&1 \
    || { tail -20 gpurun_out/bench_tlog${r}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_tlog${r}_$TAG.log | cut -c1-300
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlog_$TAG -o run --output-format csv \
  -- python3 bench.py --type tlog --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tlog_$TAG.log 2>&1 || exit 1
echo "tlog quick done"
