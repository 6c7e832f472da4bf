set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
for v in new room8 cp0; do
  L=$PWD/jylis_amd/libjylis_gpu.so; E=""
  [ $v = room8 ] && L=$PWD/jylis_amd/_ab/libjylis_room8.so
  [ $v = cp0 ] && E="JY_COPY_THREADS=0"
  env $E JY_LIB=$L timeout -k 10 300 python3 bench.py --type ujson --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/uj5_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/uj5_${v}_$rep.log; exit 1; }
  echo "$v $rep $(grep -h '^{' gpurun_out/uj5_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['per_converge']['touched_cloud'], d['roofline']['converge_ms_avg'], d['verified_sampled_docs'])")"
done
done
