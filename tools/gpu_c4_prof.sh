#!/bin/bash
# C4 (multi-scale 1280x720) and C5-shaped single-scale 720p: bench lines + rocprofv3 kernel stats.
# usage: tools/gpu_c4_prof.sh TAG
set -o pipefail
TAG=${1:-c4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python bench.py --frame 720x1280 --precise --batch 8 --steps 5 --warmup 2 > $OUT/bench_c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --frame 720x1280 --batch 21 --steps 10 --warmup 2 > $OUT/bench_c5.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --frame 720x1280 --precise --batch 8 --steps 3 --warmup 1 --no-profile > $OUT/prof_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --frame 720x1280 --batch 21 --steps 3 --warmup 1 --no-profile > $OUT/prof_c5.log 2>&1 || exit $?
