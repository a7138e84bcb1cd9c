#!/bin/bash
# Rehearsal of the N>1 bench control flow on a 1-GPU box: 2 ranks share device 0 (OP_BENCH_DEVICE=0).
# RCCL refuses two ranks on one GPU, so the gather falls back to the labelled TCP gather; the
# driver's 8-GPU run (one rank per GPU) takes the RCCL path.  The sharded frames, barriers,
# max-over-ranks timing and the JSON line are the ones the driver's run uses.
set -o pipefail
mkdir -p gpurun_out
OP_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/rehearse_n2.log 2>&1
