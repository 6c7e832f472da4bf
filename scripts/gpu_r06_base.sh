#!/bin/bash
# Round-6 baseline of the UJSON row: the bench line at --warmup 2 and 20
# (flatness), a kernel trace, and FETCH / WRITE PMC passes of steady
# converges.  Every GPU step under its own limit, chained with &&.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06base}
W=${WARMUPS:-2 20}
for w in $W; do
  timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup $w --no-cpu-baseline \
    > gpurun_out/bench_ujson_w${w}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_ujson_w${w}_$TAG.log; exit 1; }
  echo "w=$w $(grep -h '^{' gpurun_out/bench_ujson_w${w}_$TAG.log | grep -o '"converge_ms_avg[^,]*\|"frac[^,]*\|verified_sampled_docs[^,]*\|"touched_el[^,]*' | tr '\n' ' ')"
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ujson_$TAG -o run --output-format csv -- \
    python3 bench.py --type ujson --steps 8 --warmup 6 --no-cpu-baseline > gpurun_out/prof_ujson_$TAG.log 2>&1 \
    || { tail -20 gpurun_out/prof_ujson_$TAG.log; exit 1; }
  echo "prof ok"
fi
if [ -n "${PMC:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_ujson_${c}_$TAG -o run --output-format csv -- \
      python3 bench.py --type ujson --steps 4 --warmup 6 --no-cpu-baseline > gpurun_out/pmc_ujson_${c}_$TAG.log 2>&1 \
      || { tail -20 gpurun_out/pmc_ujson_${c}_$TAG.log; exit 1; }
    echo "pmc $c ok"
  done
fi
echo "base done"
