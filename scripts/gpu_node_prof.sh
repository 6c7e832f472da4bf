#!/bin/bash
# Kernel trace of the node TREG line (S = 1 over RCCL) and the timeline of
# one timed call (marker: the call's first ingest kernel).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
MARK=${MARK:-k_nd1_head}
for v in 0 1; do  # A/B: S = 1 read in place (0) vs through the regroup + self exchange (1)
  JY_NODE_REGROUP_ONE=$v timeout -k 10 300 python bench.py --type treg --node --steps 8 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_treg_node_regroup${v}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_treg_node_regroup${v}_$TAG.log; exit 1; }
  echo "regroup=$v $(grep -h '^{' gpurun_out/bench_treg_node_regroup${v}_$TAG.log | grep -o '"ms_per_step[^,]*\|verified[^,]*' | tr '\n' ' ')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_node_$TAG -o run --output-format csv -- \
  python3 bench.py --type treg --node --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_treg_node_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_treg_node_$TAG.log; exit 1; }
grep -h '^{' gpurun_out/prof_treg_node_$TAG.log | cut -c1-400
kt=$(find gpurun_out/prof_treg_node_$TAG -name '*kernel_trace.csv' | head -1)
python3 scripts/ktimeline.py "$kt" "$MARK" -3 > gpurun_out/timeline_treg_node_$TAG.txt
tail -3 gpurun_out/timeline_treg_node_$TAG.txt
echo "node prof done"
