#!/bin/bash
# kernel traces of the bench for each conv family: tools/gpu_trace_algo.sh BATCH mode...
set -o pipefail
B=$1; shift
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  mkdir -p $GRAFT_REPO_ROOT/gpurun_out/tra_$m
  OP_HALO_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tra_$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --batch $B --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/tra_$m/bench.log 2>&1 || exit $?
done
