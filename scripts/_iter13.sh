set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/uj_diag.py --reps 7 > gpurun_out/ujdiag.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ujdiag.log | tail -60
exit $rc
