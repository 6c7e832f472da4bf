#!/bin/bash
# Round evidence, part 2: headline bench with both CPU baselines, then
# rocprofv3 kernel-trace stats of the headline and of every mode.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
echo "prof headline ok"
TAG=r01 STEPS=8 bash scripts/gpu_prof_modes.sh
