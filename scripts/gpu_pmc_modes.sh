#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel for bench modes (one PMC pass per counter).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
for m in ${MODES:-treg tlog}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 ${STEP_TIMEOUT:-400} rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_${m}_${c}_$TAG -o run --output-format csv \
      -- python3 bench.py --type $m --steps 3 --warmup 1 --batches 2 --no-cpu-baseline ${EXTRA:-} > gpurun_out/pmc_${m}_$c.log 2>&1
    rc=$?; echo "pmc $m $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
echo "pmc modes done"
