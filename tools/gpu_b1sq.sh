#!/bin/bash
# One SQ PMC pass (kernel trace only) over the one-frame workload: wait / issue counters per kernel,
# for the conv_m16q stall.  usage: tools/gpu_b1sq.sh TAG  (env such as
# OP_M16Q_BPF=1 passes through to the bench)
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/b1sq_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 1 --steps 20 --warmup 5 --no-cpu-baseline --no-variants --no-profile > $OUT/bench.log 2>&1
