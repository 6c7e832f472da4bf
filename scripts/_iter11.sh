set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in head 609d880 9ca9ccd new; do
  L=$PWD/jylis_amd/libjylis_gpu.so; [ $v != new ] && L=$PWD/jylis_amd/_ab/libjylis_$v.so
  echo "== $v"
  JY_LIB=$L timeout -k 10 280 python3 -u tools/uj_repro.py --reps 5 > gpurun_out/ujrepro_$v.log 2>&1; rc=$?
  grep -E '^rep|distinct' gpurun_out/ujrepro_$v.log
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ujrepro_$v.log; exit 1; }
done
