#!/bin/bash
# The config-4 full-size TLOG pin for each library variant (LIBS: "new" = the
# tree's build, X = jylis_amd/_ab/libjylis_X.so).  A test failure goes on to
# the next variant; a time limit, abort or fault ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${LIBS:-new}; do
  if [ $v = new ]; then L=$PWD/jylis_amd/libjylis_gpu.so; else L=$PWD/jylis_amd/_ab/libjylis_$v.so; fi
  JY_LIB=$L timeout -k 10 500 python -u -m pytest "tests/test_fullsize_gpu.py::test_tlog_config4_fullsize" -m gpu -x -q \
    --timeout 480 --timeout-method thread > gpurun_out/pytest_fs_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -1 gpurun_out/pytest_fs_$v.log)"
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
