#!/bin/bash
# Counter campaign: FETCH/WRITE calibration (tools/mb_fetch; SKIP_CAL=1 skips
# it), then per bench mode (MODES, extra bench arguments in BENCH_ARGS) an SQ
# pass and separate FETCH_SIZE / WRITE_SIZE passes.  Every
# pass is its own profiled process under its own limit (rocprofv3 does not
# split counters over passes).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
run() {  # dir counters cmd...
  local d=$1 c=$2; shift 2
  timeout -k 10 ${STEP_TIMEOUT:-300} rocprofv3 --pmc $c --kernel-trace -d gpurun_out/$d -o run --output-format csv -- "$@" \
    > gpurun_out/$d.log 2>&1
  local rc=$?; echo "$d rc=$rc"; return $rc
}
if [ -z "${SKIP_CAL:-}" ]; then
  run pmc_cal_fetch_$TAG FETCH_SIZE ./tools/mb_fetch || exit 1
  run pmc_cal_write_$TAG WRITE_SIZE ./tools/mb_fetch || exit 1
fi
for m in ${MODES:-tlog ujson treg}; do
  B="python3 bench.py --type $m --steps 3 --warmup 1 --batches 2 --no-cpu-baseline ${BENCH_ARGS:-}"
  run pmc_${m}_sq_$TAG "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" $B || exit 1
  run pmc_${m}_fetch_$TAG FETCH_SIZE $B || exit 1
  run pmc_${m}_write_$TAG WRITE_SIZE $B || exit 1
done
python3 scripts/pmc_summary.py gpurun_out/pmc_summary_$TAG.json gpurun_out/pmc_*_$TAG
