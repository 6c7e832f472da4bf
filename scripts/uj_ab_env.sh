#!/bin/bash
# in-box A/B by environment: default vs $ABENV=1 (UJSON bench lines,
# alternated twice), after the UJSON GPU parity tests
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
ABENV=${ABENV:-JY_UJ_SAFE_GRID}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "ujson" \
  > gpurun_out/pytest_ujenv.log 2>&1 || { tail -40 gpurun_out/pytest_ujenv.log; exit 1; }
tail -1 gpurun_out/pytest_ujenv.log
for r in 1 2; do
  for v in new alt; do
    if [ $v = alt ]; then export $ABENV=1; else unset $ABENV; fi
    timeout -k 10 300 python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ujenv_${v}_$r.log 2>&1 || exit 1
    echo "== $v $r $(grep -h '^{' gpurun_out/ujenv_${v}_$r.log | grep -o '"converge_ms_avg[^,]*\|verified[^,]*' | tr '\n' ' ')"
  done
done
unset $ABENV
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ujenv -o run --output-format csv -- python3 bench.py --type ujson --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ujenv.log 2>&1 || exit 1
echo done
