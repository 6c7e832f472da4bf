#!/bin/bash
# Kernel trace of the routed TREG step at N = 1 (partition, exchange to
# itself, receiver merge): where the routed step's time goes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tregroute_$TAG -o run --output-format csv \
  -- python3 bench.py --type treg --route --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_tregroute_$TAG.log 2>&1 || exit 1
grep -h '^{' gpurun_out/prof_tregroute_$TAG.log | cut -c1-300
echo "route prof done"
