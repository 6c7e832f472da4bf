#!/bin/bash
# full GPU suite, then the e2e ingest line (host key strings through the
# C-ABI) and its kernel stats
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02k}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py --type e2e --steps 8 --warmup 2 > gpurun_out/bench_e2e_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_e2e_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_e2e_$TAG.log | grep -o '"value[^,]*\|"ms_per_step[^,]*\|"host_intern_ms[^,]*' | tr '\n' ' '; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e_$TAG -o run --output-format csv -- python3 bench.py --type e2e --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_e2e_$TAG.log 2>&1 || exit 1
echo done
