#!/bin/bash
# Kernel trace + stats of the batch-1 latency workload (one 368x368 frame per step).  usage: tools/gpu_b1prof.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/b1prof_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 1 --steps 40 --warmup 5 --no-cpu-baseline --no-variants --no-profile "$@" > $OUT/bench.log 2>&1 || exit $?
echo done
