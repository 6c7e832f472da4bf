#!/bin/bash
# UJSON parity tests, bench line + kernel stats, and the per-tile probe build
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-uj}
timeout -k 10 600 python -u -m pytest tests/test_parity_ujson.py tests/test_ujson_write_gpu.py tests/test_ujson_doc.py tests/test_route_csr_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ujson_$TAG -o run --output-format csv -- python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ujson_$TAG.log 2>&1 || exit 1
grep -h '^{' gpurun_out/bench_ujson_$TAG.log | cut -c1-200
python3 scripts/kstats.py gpurun_out/prof_ujson_$TAG/run_kernel_stats.csv 9 | grep k_uj
if [ -n "${PROBE:-}" ]; then
  rm -f gpurun_out/ujprobe_$TAG.bin
  JY_LIB=$PWD/jylis_amd/abx/libjylis_ujprobe.so JY_UJ_PROBE_OUT=gpurun_out/ujprobe_$TAG.bin timeout -k 10 400 python bench.py --type ujson --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ujprobe_$TAG.log 2>&1 || exit 1
  python3 tools/uj_probe_report.py gpurun_out/ujprobe_$TAG.bin | head -8
fi
