#!/bin/bash
# Node bench lines on one MI355X: TREG through the node (S = 1 over RCCL,
# S = 2 copy fabric), the PNCOUNT routed phase rehearsed at N = 1 (native
# node block converge + CounterRouter), each step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
run() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python bench.py "$@" > gpurun_out/bench_${name}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${name}_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${name}_$TAG.log | cut -c1-600
}
run treg_node 400 --type treg --node --steps 8 --warmup 2 --no-cpu-baseline
run treg_node2 400 --type treg --node --node-shards 2 --steps 8 --warmup 2 --no-cpu-baseline
run pncount_route 600 --route --steps 4 --warmup 1 --batches 2 --no-cpu-baseline
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_node_$TAG -o run --output-format csv -- python3 bench.py --type treg --node --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_treg_node_$TAG.log 2>&1 || exit 1
fi
echo "node bench done"
