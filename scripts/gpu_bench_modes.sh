#!/bin/bash
# Per-mode bench lines (and optionally a rocprofv3 kernel-trace summary of
# each).  MODES="treg tlog ..."; EXTRA="--route" etc.; PROF=1 adds --stats.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
for m in ${MODES:-treg}; do
  name=${m}${SUFFIX:-}
  timeout -k 10 400 python bench.py --type $m --steps ${STEPS:-8} --warmup 2 --batches 2 --no-cpu-baseline ${EXTRA:-} \
    > gpurun_out/bench_${name}_$TAG.log 2>&1 || exit $?
  grep -h '^{' gpurun_out/bench_${name}_$TAG.log | cut -c1-600
  if [ "${PROF:-0}" = 1 ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${name}_$TAG -o run --output-format csv -- \
      python3 bench.py --type $m --steps ${STEPS:-8} --warmup 2 --batches 2 --no-cpu-baseline ${EXTRA:-} \
      > gpurun_out/prof_${name}_$TAG.log 2>&1 || exit $?
    f=$(find gpurun_out/prof_${name}_$TAG -name '*kernel_stats.csv' | head -1)
    cp "$f" gpurun_out/${name}_kernel_stats_$TAG.csv
    cut -d, -f1-4 gpurun_out/${name}_kernel_stats_$TAG.csv | head -12
  fi
done
echo "bench modes done"
