#!/bin/bash
# Kernel-time A/B aid: tools/kstats.sh TAG "ENV=a ENV2=b" [bench args...] -> gpurun_out/kst_TAG_<n>/
# (rocprofv3 --kernel-trace --stats of a short default bench run under the given environment;
# summarise with tools/kstats_sum.py PATTERN gpurun_out/kst_*)
set -o pipefail
TAG=$1; ENVS=$2; shift 2
n=0; while [ -e $GRAFT_REPO_ROOT/gpurun_out/kst_${TAG}_$n ]; do n=$((n + 1)); done
O=$GRAFT_REPO_ROOT/gpurun_out/kst_${TAG}_$n; mkdir -p $O
echo "$ENVS" > $O/env.txt
cd /tmp && export TMPDIR=/tmp
env $ENVS timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-variants --no-profile "$@" > $O/bench.log 2>&1
