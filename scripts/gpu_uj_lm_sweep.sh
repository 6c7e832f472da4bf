#!/bin/bash
# UJSON: the config-5 line at several promotion thresholds of the in-place
# layout (JY_UJ_LONG_MIN; 0 = the regular path only), one bench process each.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for lm in ${LMS:-32 64 512 0}; do
  JY_UJ_LONG_MIN=$lm timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup ${W:-6} --no-cpu-baseline \
    > gpurun_out/lm_$lm.log 2>&1 || { tail -20 gpurun_out/lm_$lm.log; exit 1; }
  echo "lm=$lm $(grep -h '^{' gpurun_out/lm_$lm.log | grep -o '"converge_ms_avg[^,]*\|"touched_el[^,]*\|"inplace_docs[^,]*\|"promoted[^,]*\|"demoted[^,]*' | tr '\n' ' ')"
done
