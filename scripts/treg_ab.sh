# A/B of TREG kernel variants built into jylis_amd/_ab/treg_*.so (JY_LIB selects the library)
mkdir -p gpurun_out
for f in ${TESTS_AB:-jylis_amd/_ab/treg_*.so}; do
  n=$(basename $f .so)
  JY_LIB=$PWD/$f timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_treg.py -m gpu > gpurun_out/ab_$n.log 2>&1
  rc=$?; echo "$n test rc=$rc $(tail -1 gpurun_out/ab_$n.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
for rep in ${REPS:-1 2}; do
for f in jylis_amd/_ab/treg_*.so; do
  n=$(basename $f .so)
  JY_LIB=$PWD/$f timeout -k 10 300 python bench.py --type treg --steps 20 --warmup 2 --batches 4 --no-cpu-baseline > gpurun_out/abb_$n.log 2>&1 || exit $?
  python - gpurun_out/abb_$n.log $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]; print(sys.argv[2], "kernel_ms %.4f frac %.4f wf %.3f" % (r["kernel_ms_avg"], r["frac"], d.get("winner_fraction", 0)))
PY
done
done
# shard-size sensitivity of each variant
[ "${SKIP_BIG:-0}" = 1 ] && exit 0
for f in jylis_amd/_ab/treg_*.so; do
  n=$(basename $f .so)
  JY_LIB=$PWD/$f timeout -k 10 400 python bench.py --type treg --keys ${BIGKEYS:-67108864} --steps ${BIGSTEPS:-10} --warmup 2 --batches ${BIGBATCHES:-2} --no-cpu-baseline > gpurun_out/abb_big_$n.log 2>&1 || exit $?
  grep -h '^{' gpurun_out/abb_big_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("big '$n'", d["units_per_step_per_gpu"], "kernel_ms %.4f frac %.4f" % (r["kernel_ms_avg"], r["frac"]))'
done
