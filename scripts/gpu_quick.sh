#!/bin/bash
# A subset of the GPU suite (FILES) plus, with PROF=1, the node TREG timeline.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
FILES=${FILES:-tests/test_keys_gpu.py tests/test_parity_tlog.py tests/test_parity_ujson.py tests/test_node_gpu.py}
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_quick_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_quick_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_quick_$TAG.log
if [ -n "${PROF:-}" ]; then bash scripts/gpu_node_prof.sh || exit 1; fi
echo "quick done"
