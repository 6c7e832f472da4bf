#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace.  Every GPU
# step has its own time limit; a fault / abort / timeout ends the session.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() {  # $1 = exit code of the previous GPU step
  case "$1" in
    0|1) return 0 ;;   # pass / ordinary test failure
    *) echo "GPU step ended with $1: stopping" ; exit "$1" ;;
  esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -5 gpurun_out/pytest_gpu.log
  stop_on_fault $rc
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log; tail -3 gpurun_out/bench.log
  stop_on_fault $rc
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
    -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc" >> gpurun_out/prof.log; tail -3 gpurun_out/prof.log
  stop_on_fault $rc
fi
echo "session done"
