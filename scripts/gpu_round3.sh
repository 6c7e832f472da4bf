#!/bin/bash
# Round evidence refresh after the routing/UJSON changes: per-mode lines and
# kernel stats of the modes whose kernels changed.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in gcount treg tlog ujson; do
  timeout -k 10 400 python bench.py --type $m --steps 8 --warmup 1 --batches 2 > gpurun_out/bench_$m.log 2>&1 || exit $?
  grep -h '^{' gpurun_out/bench_$m.log | cut -c1-160
done
timeout -k 10 400 python bench.py --type treg --route --steps 8 --warmup 1 --batches 2 --no-cpu-baseline > gpurun_out/bench_treg_route.log 2>&1 || exit $?
TAG=r01 STEPS=8 MODES="treg ujson" bash scripts/gpu_prof_modes.sh
