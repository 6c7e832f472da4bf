#!/bin/bash
# A/B of the TREG first-occurrence claim (JY_CLAIM_MODE builds in jylis_amd/abx/):
# the shipped library (mode 2) against per-lane atomics (1) and no claim (0,
# unsafe: cost reference only).  One bench line each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in main abx/libjylis_claim0.so; do
  if [ $v = main ]; then unset JY_LIB; else export JY_LIB=$PWD/jylis_amd/$v; fi
  timeout -k 10 300 python bench.py --type treg --steps 10 --warmup 2 --batches 2 --no-cpu-baseline \
    > gpurun_out/claim_ab.log 2>&1 || exit $?
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/claim_ab.log') if l.startswith('{')][0]; print('$v', round(d['roofline']['kernel_ms_avg']*1e3,1), 'us', round(d['roofline']['frac'],3))"
done
