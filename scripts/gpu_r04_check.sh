#!/bin/bash
# Round-4 change check: smoke, the TREG / TLOG / node tests, the TREG (block +
# keyed), TLOG and routed PNCOUNT lines, and a TLOG kernel trace.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r04}
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python -u -m pytest tests/test_parity_treg.py tests/test_parity_tlog.py tests/test_node_gpu.py \
  tests/test_write_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_chk_$TAG.log 2>&1 \
  || { tail -30 gpurun_out/pytest_chk_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_chk_$TAG.log
run() {  # name limit args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > gpurun_out/bench_${name}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${name}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${name}_$TAG.log | cut -c1-200
}
run treg 400 --type treg --steps 10 --warmup 3 --no-cpu-baseline
run tlog 400 --type tlog --steps 8 --warmup 2 --no-cpu-baseline
run pncount_route 500 --route --steps 4 --warmup 1 --batches 2 --no-cpu-baseline
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlog_$TAG -o run --output-format csv \
  -- python3 bench.py --type tlog --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tlog_$TAG.log 2>&1 || exit 1
echo "r04 check done"
