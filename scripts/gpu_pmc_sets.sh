#!/bin/bash
# rocprofv3 counter passes over one bench mode: each PASS is a space-separated
# counter group ("A B,C D" = two passes), run as its own profiled process with
# its own time limit.  Output: gpurun_out/pmcset_<mode>_<i>_<TAG>/
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
MODE=${MODE:-tlog}
IFS=',' read -ra PASSES <<< "${PASSES:-SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS,FETCH_SIZE,WRITE_SIZE}"
i=0
for pass in "${PASSES[@]}"; do
  timeout -k 10 ${STEP_TIMEOUT:-400} rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/pmcset_${MODE}_${i}_$TAG -o run \
    --output-format csv -- python3 bench.py --type $MODE --steps 3 --warmup 1 --no-cpu-baseline ${EXTRA:-} \
    > gpurun_out/pmcset_${MODE}_$i.log 2>&1
  rc=$?; echo "pmc pass $i ($pass) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  i=$((i + 1))
done
echo "pmc sets done"
