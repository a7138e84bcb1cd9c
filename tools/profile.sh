#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root):
#   tools/profile.sh <tag> [bench args...]
# 1) kernel trace + stats; 2) FETCH_SIZE pass; 3) WRITE_SIZE pass (separate PMC passes, kernel trace only).
set -o pipefail
TAG=${1:-r01}; shift
ARGS="$@"
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants $ARGS > $OUT/bench_stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-profile $ARGS > $OUT/bench_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-profile $ARGS > $OUT/bench_write.log 2>&1 || exit $?
