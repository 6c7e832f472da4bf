#!/bin/bash
# TREG at 64M keys on one GPU (<true> kernel) and a gloo world-2 rehearsal of
# the default (routed PNCOUNT) bench on one GPU
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python bench.py --type treg --keys 67108864 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_treg64m_r02.log 2>&1 || { tail -20 gpurun_out/bench_treg64m_r02.log; exit 1; }
grep -h '^{' gpurun_out/bench_treg64m_r02.log | cut -c1-600
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --backend gloo --keys 1048576 --steps 3 --warmup 1 --batches 2 --no-cpu-baseline > gpurun_out/bench_pn_gloo2_r02.log 2>&1 || { tail -20 gpurun_out/bench_pn_gloo2_r02.log; exit 1; }
grep -h '^{' gpurun_out/bench_pn_gloo2_r02.log | cut -c1-600
