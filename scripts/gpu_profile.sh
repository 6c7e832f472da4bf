#!/bin/bash
# rocprofv3 evidence for the bench kernel: kernel-trace stats, then one PMC
# pass per counter (FETCH_SIZE, WRITE_SIZE).  Each GPU step time-limited;
# any fault ends the session.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS="--steps 3 --warmup 1 --batches 2 --no-cpu-baseline ${BENCH_ARGS:-}"
run() {  # name, then the command
  local name=$1; shift
  timeout -k 10 ${STEP_TIMEOUT:-500} "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/$name.log
  [ $rc -eq 0 ] || exit $rc
}
run prof_stats rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py $ARGS
run pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- python3 bench.py $ARGS
run pmc_write rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- python3 bench.py $ARGS
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG k_block_max ${CELLS:-2147483648} gpurun_out/pmc_traffic_$TAG.json
echo "profile done"
