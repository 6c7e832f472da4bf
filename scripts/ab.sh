#!/bin/bash
# In-box A/B of one bench line over library variants (JY_LIB), alternated
# REPS times; prints the chosen JSON fields of each run.
# usage: ARGS="--type treg --route" FIELDS="ms_per_step step_ms_avg_events" scripts/ab.sh new head rt1 ...
# ("new" = jylis_amd/libjylis_gpu.so, X = jylis_amd/_ab/libjylis_X.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    if [ $v = new ]; then L=$PWD/jylis_amd/libjylis_gpu.so; else L=$PWD/jylis_amd/_ab/libjylis_$v.so; fi
    log=gpurun_out/ab_${TAG}_${v}_${rep}.log
    JY_LIB=$L timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline > $log 2>&1 || { tail -20 $log; exit 1; }
    line=$(grep -h '^{' $log)
    out="$v $rep"
    for f in ${FIELDS:-ms_per_step}; do out="$out $f=$(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('$f', d.get('roofline', {}).get('$f')))")"; done
    echo "$out"
  done
done
