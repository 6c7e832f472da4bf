set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base ab; do
  if [ $v = ab ]; then export JY_LIB=$PWD/jylis_amd/abx/libjylis_tlab.so; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tlab_$v -o run --output-format csv -- python3 bench.py --type tlog --steps 20 --warmup 2 --batches 4 --no-cpu-baseline > gpurun_out/tlab_$v.log 2>&1 || exit 1
  echo "== $v"; grep -h '^{' gpurun_out/tlab_$v.log | cut -c1-300
  python3 scripts/kstats.py gpurun_out/prof_tlab_$v/run_kernel_stats.csv 6
done
