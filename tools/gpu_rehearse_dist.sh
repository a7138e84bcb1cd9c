#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks share cuda:0, gloo collectives on the CPU
# (the driver's 8-GPU run uses RCCL, one rank per GPU).
set -o pipefail
mkdir -p gpurun_out
OP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/rehearse_n2.log 2>&1
