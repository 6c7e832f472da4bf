#!/bin/bash
# Round-6 TLOG row: parity suites (SKIP_TESTS=1 skips; FULL=1 adds the
# config-4 full-size pin), the bench line at --warmup 2 and 20, a kernel
# trace (PROF=1) and FETCH / WRITE PMC passes of the timed converges (PMC=1).
# Every GPU step under its own limit, chained with &&.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06tl}
if [ -z "${SKIP_TESTS:-}" ]; then
  T="tests/test_parity_tlog.py tests/test_tlog_write_gpu.py tests/test_arena_gpu.py tests/test_route_csr_gpu.py tests/test_docs_converge.py"
  [ -n "${FULL:-}" ] && T="$T tests/test_fullsize_gpu.py::test_tlog_config4_fullsize"
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_tlog_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_tlog_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_tlog_$TAG.log
fi
for w in ${WARMUPS:-2}; do
  timeout -k 10 400 python3 bench.py --type tlog --steps 8 --warmup $w --no-cpu-baseline \
    > gpurun_out/bench_tlog_w${w}_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_tlog_w${w}_$TAG.log; exit 1; }
  echo "w=$w $(grep -h '^{' gpurun_out/bench_tlog_w${w}_$TAG.log | grep -o '"ms_per_step[^,]*\|"converge_ms_avg[^,]*\|"frac[^,]*\|verified_sampled_keys[^,]*\|"spills_compactions[^]]*' | tr '\n' ' ')"
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlog_$TAG -o run --output-format csv \
    -- python3 bench.py --type tlog --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tlog_$TAG.log 2>&1 \
    || { tail -20 gpurun_out/prof_tlog_$TAG.log; exit 1; }
  python3 scripts/kstats.py gpurun_out/prof_tlog_$TAG/run_kernel_stats.csv 8
fi
if [ -n "${PMC:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_tlog_${c}_$TAG -o run --output-format csv -- \
      python3 bench.py --type tlog --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_tlog_${c}_$TAG.log 2>&1 \
      || { tail -20 gpurun_out/pmc_tlog_${c}_$TAG.log; exit 1; }
    echo "pmc $c ok"
  done
  python3 scripts/pmc_converge.py gpurun_out/pmc_tlog_$TAG.json gpurun_out/pmc_tlog_FETCH_SIZE_$TAG \
    gpurun_out/pmc_tlog_WRITE_SIZE_$TAG k_tlog_prep 3 4
fi
echo "tlog done"
