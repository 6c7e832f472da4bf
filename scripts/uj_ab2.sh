#!/bin/bash
# in-box A/B, alternating: default build vs $AB, bench lines only
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
AB=${AB:-jylis_amd/abx/libjylis_base.so}
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export JY_LIB=$PWD/$AB; else unset JY_LIB; fi
    timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ujab2_${v}_$r.log 2>&1 || exit 1
    echo "== $v $r $(grep -h '^{' gpurun_out/ujab2_${v}_$r.log | grep -o '"converge_ms_avg[^,]*')"
  done
done
