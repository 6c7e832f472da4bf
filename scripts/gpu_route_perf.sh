#!/bin/bash
# routing parity tests, then routed vs plain TREG / TLOG / UJSON step times (1 GPU)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-rp}
timeout -k 10 500 python -u -m pytest tests/test_route_csr_gpu.py tests/test_route_gpu.py tests/test_route_dist_gpu.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for m in ${MODES:-treg tlog ujson}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${m}_route_$TAG -o run --output-format csv \
    -- python3 bench.py --type $m --route --steps 8 --warmup 2 --batches 3 --no-cpu-baseline > gpurun_out/bench_${m}_route_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${m}_route_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${m}_route_$TAG.log | cut -c1-260
  python3 scripts/kstats.py gpurun_out/prof_${m}_route_$TAG/run_kernel_stats.csv 8
done
