#!/bin/bash
# Round 4: PMC evidence for C4's default two-pass map resize (resize_cubic_f32_up + _planar_mean):
# kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes and one SQ pass on the C4 workload, each a
# run of its own (kernel trace only).
set -o pipefail
bash tools/profile.sh r04c4 --precise --frame 720x1280 || exit $?
bash tools/sq_counters.sh r04c4 --precise --frame 720x1280 || exit $?
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/sq2_r04c4; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $O -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-profile > $O/bench.log 2>&1 || exit $?
echo done
