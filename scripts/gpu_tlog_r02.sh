#!/bin/bash
# TLOG parity tests, the TLOG bench line and its kernel trace
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r02t}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "tlog or host" \
  > gpurun_out/pytest_tlog_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_tlog_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_tlog_$TAG.log
timeout -k 10 400 python bench.py --type tlog --steps 8 --warmup 2 > gpurun_out/bench_tlog_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_tlog_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/bench_tlog_$TAG.log | grep -o '"ms_per_step[^,]*\|"frac[^,]*\|"converge_ms_avg[^,]*\|verified[^,]*' | tr '\n' ' '; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlog_$TAG -o run --output-format csv -- python3 bench.py --type tlog --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tlog_$TAG.log 2>&1 || exit 1
echo done
