#!/bin/bash
# Round-3 profile of the default bench workload (kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes,
# tools/profile.sh) and, with AB set, an interleaved A/B (tools/ab_lib.py) in the same call.
# usage: [AB="base NAME=VAL"] tools/gpu_prof3.sh TAG
set -o pipefail
TAG=$1
bash tools/profile.sh $TAG || exit $?
if [ -n "$AB" ]; then
  mkdir -p gpurun_out/ab_$TAG
  timeout -k 10 900 python3 -u tools/ab_lib.py ${ABR:-3} $AB > gpurun_out/ab_$TAG/ab.log 2>&1 || exit $?
fi
