#!/bin/bash
# UJSON: parity tests of the default build, then an in-box A/B of the bench
# line (default library vs JY_LIB=$AB, alternated twice), each step under its
# own limit.  PROBE=1 adds the per-tile clocks of a JY_UJ_PROBE build.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03}
AB=${AB:-jylis_amd/_ab/libjylis_old.so}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_parity_ujson.py tests/test_ujson_doc.py tests/test_ujson_write_gpu.py \
    tests/test_docs_converge.py tests/test_route_csr_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_uj_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_uj_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_uj_$TAG.log
fi
for rep in 1 2; do
  for v in new ab; do
    if [ $v = ab ]; then L=$PWD/$AB; else L=$PWD/jylis_amd/libjylis_gpu.so; fi
    JY_LIB=$L timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline \
      > gpurun_out/ujab_${v}_${rep}_$TAG.log 2>&1 || { tail -20 gpurun_out/ujab_${v}_${rep}_$TAG.log; exit 1; }
    echo "$v $rep $(grep -h '^{' gpurun_out/ujab_${v}_${rep}_$TAG.log | grep -o '"converge_ms_avg[^,]*\|"frac[^,]*\|verified_sampled_docs[^,]*' | tr '\n' ' ')"
  done
done
if [ -n "${PROBE:-}" ]; then
  rm -f gpurun_out/ujprobe_$TAG.bin
  JY_LIB=$PWD/jylis_amd/_ab/libjylis_probe.so JY_UJ_PROBE_OUT=gpurun_out/ujprobe_$TAG.bin timeout -k 10 300 \
    python3 bench.py --type ujson --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ujprobe_$TAG.log 2>&1 || exit 1
  python3 tools/uj_probe_report.py gpurun_out/ujprobe_$TAG.bin
fi
echo "ujson ab done"
