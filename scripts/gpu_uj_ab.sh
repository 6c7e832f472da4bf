#!/bin/bash
# UJSON A/B on one box: bench with the small-document kernel and without
# (JY_UJ_NOSMALL), then a kernel trace of the default form.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02v}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "ujson" > gpurun_out/pytest_uj_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_uj_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_uj_$TAG.log
fi
timeout -k 10 400 python bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ujson_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_ujson_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_ujson_$TAG.log | grep -o '"frac[^,]*,\|"converge_ms_avg[^,]*,\|verified[^,]*,'
JY_UJ_NOSMALL=1 timeout -k 10 400 python bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ujson_nosmall_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_ujson_nosmall_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_ujson_nosmall_$TAG.log | grep -o '"frac[^,]*,\|"converge_ms_avg[^,]*,\|verified[^,]*,'
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ujson_$TAG -o run --output-format csv -- python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ujson_$TAG.log 2>&1 || exit 1
fi
echo "gpu_uj_ab done"
