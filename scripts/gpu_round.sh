#!/bin/bash
# Round-end evidence on one MI355X: the full GPU parity suite, the headline
# bench (with cpu_baseline) and every per-mode bench line, then rocprofv3
# stats of the headline and of each mode.  Each step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export JY_PROGRESS=$PWD/gpurun_out/progress_${TAG:-r04}.log
TAG=${TAG:-r03}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
fi
if [ -z "${SKIP_HEAD:-}" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_$TAG.log | cut -c1-400
fi
# UJSON warms up past its first pool compaction (sized from the state the
# setup converge built; later ones are ~50 converges apart)
wu() { [ "$1" = ujson ] && echo 6 || echo 2; }
for m in ${MODES-gcount treg tlog ujson e2e read}; do
  timeout -k 10 400 python bench.py --type $m --steps 8 --warmup $(wu $m) > gpurun_out/bench_${m}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${m}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${m}_$TAG.log | cut -c1-300
done
if [ -z "${SKIP_ROUTE:-}" ]; then
  timeout -k 10 400 python bench.py --type treg --route --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_treg_route_$TAG.log 2>&1 || exit 1
  grep -h '^{' gpurun_out/bench_treg_route_$TAG.log | cut -c1-300
fi
if [ -n "${PROF:-}" ]; then
  [ -n "${SKIP_HEAD:-}" ] || timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batches 2 --no-cpu-baseline > gpurun_out/prof_head_$TAG.log 2>&1 || exit 1
  for m in ${PMODES-gcount treg tlog ujson e2e read}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${m}_$TAG -o run --output-format csv -- python3 bench.py --type $m --steps 8 --warmup $(wu $m) --no-cpu-baseline > gpurun_out/prof_${m}_$TAG.log 2>&1 || exit 1
  done
fi
echo "round evidence done"
