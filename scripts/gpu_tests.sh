#!/bin/bash
# GPU parity suite + short per-mode bench lines.  Each GPU step runs under its
# own time limit; the first failure ends the session (no retries).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export JY_PROGRESS=$PWD/gpurun_out/progress_${TAG:-r04}.log
TAG=${TAG:-r02}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
for m in ${MODES:-}; do
  timeout -k 10 400 python bench.py --type $m --steps 8 --warmup 2 --batches 2 --no-cpu-baseline \
    > gpurun_out/bench_${m}_$TAG.log 2>&1 || exit $?
  grep -h '^{' gpurun_out/bench_${m}_$TAG.log | cut -c1-400
done
echo "gpu_tests done"
