#!/bin/bash
# Diagnostics for the default workload: kernel trace (gaps, per-layer times) + SQ and clock counter passes.
set -o pipefail
TAG=${1:-diag}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tr_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $R/gpurun_out/tr_$TAG/bench.log 2>&1 || exit $?
cd $R && bash tools/sq_counters.sh $TAG || exit $?
cd $R && bash tools/clk_counters.sh $TAG || exit $?
