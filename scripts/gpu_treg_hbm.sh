#!/bin/bash
# TREG at HBM scale (tools/treg_hbm.py): block and keyed forms per library
# variant (VARIANTS: "new" = the tree's build, X = jylis_amd/_ab/libjylis_X.so),
# at KEYS keys; each run under its own limit, chained.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-hbm}
for rep in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-new}; do
    if [ $v = new ]; then L=$PWD/jylis_amd/libjylis_gpu.so; else L=$PWD/jylis_amd/_ab/libjylis_$v.so; fi
    JY_LIB=$L timeout -k 10 150 python3 -u tools/treg_hbm.py ${KEYS:-67108864} ${STEPS:-8} > gpurun_out/treg_hbm_${TAG}_${v}_$rep.log 2>&1 \
      || { tail -20 gpurun_out/treg_hbm_${TAG}_${v}_$rep.log; exit 1; }
    echo "$v $rep: $(grep -h 'frac' gpurun_out/treg_hbm_${TAG}_${v}_$rep.log | cut -d' ' -f1-7 | tr '\n' ' ')"
  done
done
