set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
for v in new cp0; do
  E=""; [ $v = cp0 ] && E="JY_COPY_THREADS=0"
  env $E timeout -k 10 300 python3 bench.py --type ujson --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/uj8_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/uj8_${v}_$rep.log; exit 1; }
  echo "$v $rep $(grep -h '^{' gpurun_out/uj8_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['per_converge']['touched_cloud'], d['roofline']['converge_ms_avg'], d['verified_sampled_docs'])")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_tlog_it8 -o run --output-format csv -- python3 bench.py --type tlog --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tlog_it8.log 2>&1 || exit 1
grep -h '^{' gpurun_out/prof_tlog_it8.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_uj_it8 -o run --output-format csv -- python3 bench.py --type ujson --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/prof_uj_it8.log 2>&1 || exit 1
