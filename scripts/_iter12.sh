set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
JY_LIB=$PWD/jylis_amd/libjylis_gpu.so timeout -k 10 400 python3 -u tools/uj_repro.py --reps 8 > gpurun_out/ujrepro_fix.log 2>&1; rc=$?
grep -E '^rep|distinct' gpurun_out/ujrepro_fix.log
[ $rc -eq 0 ] || { tail -5 gpurun_out/ujrepro_fix.log; exit 1; }
