#!/bin/bash
# Round-6 key directory / node row: key + node + routing suites (SKIP_TESTS=1
# skips), the node TREG bench A/B (AB="new head"), and a kernel trace of the
# node call (PROF=1) with one call's timeline.  Each GPU step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06nd}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_keys_gpu.py tests/test_converge_keys_gpu.py tests/test_node_gpu.py \
    tests/test_node_shared_gpu.py tests/test_route_gpu.py tests/test_route_csr_gpu.py tests/test_host_gpu.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_node_$TAG.log 2>&1 \
    || { tail -40 gpurun_out/pytest_node_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_node_$TAG.log
fi
if [ -n "${AB:-}" ]; then
  ARGS="--type treg --node --steps 8 --warmup 2" FIELDS="ms_per_step" TAG=nd_$TAG REPS=${REPS:-2} scripts/ab.sh $AB || exit 1
fi
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_treg_node_$TAG -o run --output-format csv \
    -- python3 bench.py --type treg --node --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_treg_node_$TAG.log 2>&1 || exit 1
  python3 scripts/ktimeline.py gpurun_out/prof_treg_node_$TAG/run_kernel_trace.csv k_key_probe -3 > gpurun_out/node_timeline_$TAG.txt
  cat gpurun_out/node_timeline_$TAG.txt
fi
echo "node done"
