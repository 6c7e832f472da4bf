#!/bin/bash
# UJSON A/B: default build vs an A/B library (JY_LIB), kernel stats of each
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
AB=${AB:-jylis_amd/abx/libjylis_ujab.so}
for v in base ab; do
  if [ $v = ab ]; then export JY_LIB=$PWD/$AB; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ujab_$v -o run --output-format csv -- python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ujab_$v.log 2>&1 || exit 1
  echo "== $v"; grep -h '^{' gpurun_out/ujab_$v.log | cut -c1-160
  python3 scripts/kstats.py gpurun_out/prof_ujab_$v/run_kernel_stats.csv 9 | grep k_uj
done
