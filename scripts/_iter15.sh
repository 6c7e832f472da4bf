set -u
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_it15.log 2>&1 || { tail -30 gpurun_out/pytest_it15.log; exit 1; }
tail -1 gpurun_out/pytest_it15.log
TAG=treg15 ARGS="--type treg --steps 10 --warmup 3" FIELDS="kernel_ms_avg frac ms_per_step verified_sampled_keys" bash scripts/ab.sh head new || exit 1
TAG=tregr15 ARGS="--type treg --route --steps 10 --warmup 3" FIELDS="step_ms_avg_events ms_per_step verified_sampled_keys" bash scripts/ab.sh new || exit 1
