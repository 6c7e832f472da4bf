#!/bin/bash
# The node tests (jy_node_*) and the TREG overflow test first, then the whole
# GPU suite; each step under its own time limit, the first failure ends it.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export JY_PROGRESS=$PWD/gpurun_out/progress_${TAG:-r04}.log
TAG=${TAG:-r04}
timeout -k 10 600 python -u -m pytest tests/test_node_gpu.py tests/test_parity_treg.py -x -v --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_node_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_node_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -z "${SKIP_ALL:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_$TAG.log
fi
echo "gpu_node done"
