#!/bin/bash
# Parity tests, then each bench mode once (own time limit per step).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
fi
for m in ${MODES:-gcount treg tlog ujson}; do
  timeout -k 10 ${MODE_TIMEOUT:-400} python bench.py --type $m --steps ${STEPS:-5} --warmup 1 --batches 2 ${EXTRA:-} > gpurun_out/bench_$m.log 2>&1
  rc=$?; echo "bench $m rc=$rc" >> gpurun_out/bench_$m.log; tail -2 gpurun_out/bench_$m.log
  [ $rc -eq 0 ] || exit $rc
done
echo "modes done"
