#!/bin/bash
# UJSON parity tests, then the full GPU suite, then the UJSON bench line and
# its rocprofv3 kernel stats.  Each GPU step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02u}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "ujson" > gpurun_out/pytest_uj_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_uj_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_uj_$TAG.log
timeout -k 10 400 python bench.py --type ujson --steps 8 --warmup 2 > gpurun_out/bench_ujson_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_ujson_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_ujson_$TAG.log | cut -c1-1500
if [ -n "${FULL:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
fi
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ujson_$TAG -o run --output-format csv -- python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ujson_$TAG.log 2>&1 || exit 1
fi
echo "gpu_uj done"
