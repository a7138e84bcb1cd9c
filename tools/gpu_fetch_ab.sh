#!/bin/bash
# One FETCH_SIZE pass (kernel trace only, no other PMC or trace domain) of the default bench per
# spec, summarised per kernel by tools/fetch_sum.py.   usage: tools/gpu_fetch_ab.sh TAG spec...
# (spec: base, a library variant name (OP_LIB_VARIANT), or NAME=VALUE[,NAME=VALUE])
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/fetch_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  (
    if [ "$spec" != base ]; then
      case "$spec" in
        *=*) for kv in ${spec//,/ }; do export "$kv"; done ;;
        *) export OP_LIB_VARIANT=$spec ;;
      esac
    fi
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/$spec -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-profile \
      > $OUT/$spec.log 2>&1
  ) || exit $?
  python3 $GRAFT_REPO_ROOT/tools/fetch_sum.py $OUT/$spec >> $OUT/summary.txt || exit $?
done
