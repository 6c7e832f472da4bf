#!/bin/bash
# rocprofv3 kernel-trace stats of each bench mode (own time limit per step).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
for m in ${MODES:-gcount treg tlog ujson}; do
  timeout -k 10 ${MODE_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${m}_$TAG -o run --output-format csv \
    -- python3 bench.py --type $m --steps ${STEPS:-5} --warmup 1 --batches 2 ${EXTRA:-} > gpurun_out/prof_$m.log 2>&1
  rc=$?; echo "prof $m rc=$rc"; grep -h '^{' gpurun_out/prof_$m.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
echo "prof modes done"
