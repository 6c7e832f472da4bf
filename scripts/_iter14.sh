set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/uj_repro.py --reps 8 > gpurun_out/ujrepro_fix2.log 2>&1; rc=$?
grep -E '^rep|distinct' gpurun_out/ujrepro_fix2.log
[ $rc -eq 0 ] || { tail -5 gpurun_out/ujrepro_fix2.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_ujson_determinism_gpu.py tests/test_parity_ujson.py tests/test_ujson_doc.py tests/test_ujson_write_gpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_it14.log 2>&1 || { tail -30 gpurun_out/pytest_it14.log; exit 1; }
tail -1 gpurun_out/pytest_it14.log
JY_LIB=$PWD/jylis_amd/_ab/libjylis_head.so timeout -k 10 300 python -u -m pytest tests/test_ujson_determinism_gpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_it14_head.log 2>&1; echo "head determinism test rc=$?"; tail -2 gpurun_out/pytest_it14_head.log
