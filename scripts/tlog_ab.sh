# A/B of TLOG kernel variants built into jylis_amd/_ab/*.so (JY_LIB selects the library)
for f in jylis_amd/_ab/*.so; do
  n=$(basename $f .so)
  JY_LIB=$PWD/$f timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_tlog.py -m gpu > gpurun_out/ab_$n.log 2>&1
  rc=$?; echo "$n test rc=$rc $(tail -1 gpurun_out/ab_$n.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
  [ $rc = 0 ] || continue
  JY_LIB=$PWD/$f timeout -k 10 300 python bench.py --type tlog --steps 8 --warmup 1 --batches 2 --no-cpu-baseline > gpurun_out/abb_$n.log 2>&1 || exit $?
  python - gpurun_out/abb_$n.log $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(sys.argv[2], "ms/step %.3f converge_ms %.3f frac %.3f" % (d["ms_per_step"], d["roofline"]["converge_ms_avg"], d["roofline"]["frac"]))
PY
done
