#!/bin/bash
# TREG PMC at 8M and 64M keys (tools/treg_hbm.py, block then keyed form):
# FETCH_SIZE and WRITE_SIZE passes, each its own profiled process.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06tr}
for k in ${KEYS:-8388608 67108864}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 200 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_treg_${k}_${c}_$TAG -o run --output-format csv -- \
      python3 -u tools/treg_hbm.py $k 4 > gpurun_out/pmc_treg_${k}_${c}_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_treg_${k}_${c}_$TAG.log; exit 1; }
    echo "pmc $k $c ok"
  done
done
echo "treg pmc done"
