#!/bin/bash
# UJSON A/B: the UJSON parity suites on the default build, then the config-5
# bench line alternating builds (LIBS, JY_LIB paths; "" = the default build)
# at warmup W for ROUNDS rounds.  Every GPU step under its own limit.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ujab}
TESTS=${TESTS:-tests/test_ujson_inplace_gpu.py tests/test_parity_ujson.py tests/test_ujson_write_gpu.py tests/test_ujson_doc.py tests/test_ujson_determinism_gpu.py tests/test_docs_converge.py}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
for r in $(seq ${ROUNDS:-3}); do
  for lib in ${LIBS:-jylis_amd/_ab/libjylis_base.so default}; do
    [ "$lib" = default ] && L="" || L="$lib"
    JY_LIB="$L" timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup ${W:-6} --no-cpu-baseline \
      > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
    echo "$r $lib $(grep -h '^{' gpurun_out/bench_$TAG.log | grep -o '"converge_ms_avg[^,]*\|"ms_per_step[^,]*' | tr '\n' ' ')"
  done
done
echo "ab done"
