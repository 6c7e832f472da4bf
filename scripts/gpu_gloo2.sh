#!/bin/bash
# world-2 rehearsals of the N > 1 bench paths on one GPU (gloo: both ranks
# share the card): the default routed PNCOUNT line and the routed TREG / TLOG /
# UJSON modes; every line verifies sampled keys against their owners
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r03}
for m in ${MODES:-pncount treg tlog ujson}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2957$((RANDOM % 10)) bench.py --gpus 2 --type $m --backend gloo --keys ${KEYS:-1048576} --steps 3 \
    --warmup 1 --batches 2 --no-cpu-baseline > gpurun_out/bench_${m}_gloo2_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_${m}_gloo2_$TAG.log; exit 1; }
  grep -h '^{' gpurun_out/bench_${m}_gloo2_$TAG.log | grep -o '"value[^,]*\|"ms_per_step[^,]*\|verified[^,]*' | tr '\n' ' '; echo " $m"
done
