#!/bin/bash
# GRBM/SQ cycle counters (effective shader clock per kernel): tools/clk_counters.sh <tag> [bench args]
set -o pipefail
TAG=${1:-clk}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/clk_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile "$@" > $OUT/bench.log 2>&1
