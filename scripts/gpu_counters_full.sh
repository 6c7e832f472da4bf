#!/bin/bash
# Configs 1 and 2 pinned at full size against the oracle's digests
# (tests/test_fullsize_gpu.py::test_counter_config_fullsize), then the
# headline bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
export JY_PROGRESS=$PWD/gpurun_out/progress_counters_$TAG.log
timeout -k 10 1100 python -u -m pytest tests/test_fullsize_gpu.py -k counter -x -v --timeout 1000 --timeout-method thread \
  > gpurun_out/pytest_counters_full_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_counters_full_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_counters_full_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_head_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_head_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_head_$TAG.log | cut -c1-300
echo "counters done"
