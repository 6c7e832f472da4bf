#!/bin/bash
# TLOG tile-pass A/B: the TLOG tests on the working-tree library, then the
# bench line alternated over the library variants given (scripts/ab.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tlogab}
timeout -k 10 600 python -u -m pytest tests/test_parity_tlog.py tests/test_write_gpu.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for v in "$@"; do
  [ $v = new ] && continue
  JY_LIB=$PWD/jylis_amd/_ab/libjylis_$v.so timeout -k 10 600 python -u -m pytest tests/test_parity_tlog.py -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/pytest_${TAG}_$v.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_${TAG}_$v.log)"
done
TAG=$TAG REPS=${REPS:-2} ARGS="--type tlog --steps 8 --warmup 2" FIELDS="ms_per_step kernel_ms_avg" bash scripts/ab.sh "$@"
