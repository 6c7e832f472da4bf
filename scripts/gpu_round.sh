#!/bin/bash
# Round evidence, part 1: parity suite, headline bench, per-mode benches and
# the TREG 64M-key shard.  Every GPU step has its own limit; a fault, abort or
# timeout ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
for m in gcount treg tlog ujson; do
  timeout -k 10 400 python bench.py --type $m --steps 8 --warmup 1 --batches 2 > gpurun_out/bench_$m.log 2>&1 || exit $?
  grep -h '^{' gpurun_out/bench_$m.log | cut -c1-200
done
timeout -k 10 400 python bench.py --type treg --keys 67108864 --steps 20 --warmup 2 --batches 3 --no-cpu-baseline > gpurun_out/bench_treg64m.log 2>&1 || exit $?
grep -h '^{' gpurun_out/bench_treg64m.log | cut -c1-200
echo "round part 1 done"
