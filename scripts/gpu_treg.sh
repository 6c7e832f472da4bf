#!/bin/bash
# TREG: parity (routing, writes, parity tests), the plain / routed / overlap
# bench lines and a kernel trace of the routed step.  Each step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_route_gpu.py tests/test_route_dist_gpu.py tests/test_write_gpu.py \
    tests/test_parity_treg.py tests/test_arena_gpu.py tests/test_keys_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_treg_$TAG.log 2>&1 \
    || { tail -30 gpurun_out/pytest_treg_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_treg_$TAG.log
fi
for v in "" "--route" "--route --overlap 0.5" "--route --resolve" "--keys 67108864"; do
  n=$(echo "$v" | tr -d ' -')
  timeout -k 10 400 python bench.py --type treg $v --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_treg${n}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_treg${n}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_treg${n}_$TAG.log | cut -c1-600
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_route_$TAG -o run --output-format csv \
    -- python3 bench.py --type treg --route --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_treg_route_$TAG.log 2>&1 || exit 1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_ovl_$TAG -o run --output-format csv \
    -- python3 bench.py --type treg --route --overlap 0.5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_treg_ovl_$TAG.log 2>&1 || exit 1
fi
echo "treg done"
