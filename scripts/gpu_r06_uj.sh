#!/bin/bash
# Round 6, UJSON in-place layout: the UJSON parity suites (TESTS), then the
# config-5 bench line at each warmup of WARMUPS (flatness), optionally a
# kernel trace (PROF=1) and FETCH / WRITE PMC passes (PMC=1).  Every GPU step
# under its own limit; the first failure ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06uj}
TESTS=${TESTS:-tests/test_ujson_inplace_gpu.py tests/test_parity_ujson.py tests/test_ujson_write_gpu.py tests/test_ujson_doc.py tests/test_ujson_determinism_gpu.py tests/test_docs_converge.py}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
for w in ${WARMUPS:-2 20}; do
  timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup $w --no-cpu-baseline \
    > gpurun_out/bench_ujson_w${w}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_ujson_w${w}_$TAG.log; exit 1; }
  echo "w=$w $(grep -h '^{' gpurun_out/bench_ujson_w${w}_$TAG.log | grep -o '"converge_ms_avg[^,]*\|"frac[^,]*\|verified_sampled_docs[^,]*\|"touched_el[^,]*\|"inplace_docs[^,]*\|"demoted[^,]*\|"promoted[^,]*' | tr '\n' ' ')"
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
echo "uj done"
