#!/bin/bash
# routing tests on the GPU, then the routed bench lines (one GPU, the whole
# routed path against itself) with kernel stats of the TREG one
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02r}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "route" \
  > gpurun_out/pytest_route_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_route_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_route_$TAG.log
for m in treg tlog ujson; do
  timeout -k 10 400 python bench.py --type $m --route --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${m}_route_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${m}_route_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${m}_route_$TAG.log | grep -o '"ms_per_step[^,]*\|verified[^,]*' | tr '\n' ' '; echo " $m"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_route_$TAG -o run --output-format csv -- python3 bench.py --type treg --route --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_treg_route_$TAG.log 2>&1 || exit 1
echo done
