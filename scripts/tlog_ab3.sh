#!/bin/bash
# TLOG parity on the default build, then A/B bench + kernel stats: lane-per-key (default) vs key tiles
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_tlog.py tests/test_tlog_write_gpu.py tests/test_arena_gpu.py tests/test_route_csr_gpu.py tests/test_docs_converge.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_tlab3.log 2>&1 || { tail -30 gpurun_out/pytest_tlab3.log; exit 1; }
tail -1 gpurun_out/pytest_tlab3.log
for v in new old; do
  if [ $v = old ]; then export JY_LIB=$PWD/${AB:-jylis_amd/abx/libjylis_tltile.so}; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlab3_$v -o run --output-format csv -- python3 bench.py --type tlog --steps 20 --warmup 2 --batches 4 --no-cpu-baseline > gpurun_out/tlab3_$v.log 2>&1 || exit 1
  echo "== $v"; grep -h '^{' gpurun_out/tlab3_$v.log | cut -c1-200
  python3 scripts/kstats.py gpurun_out/prof_tlab3_$v/run_kernel_stats.csv 6
done
