#!/bin/bash
# Interleaved A/B of library variants (tools/ab_lib.py) + one SQ counter pass of the product build.
# usage: tools/gpu_ab.sh ROUNDS TAG variant...   (variants built beforehand in-tree)
set -o pipefail
R=$1; TAG=$2; shift 2
mkdir -p gpurun_out/ab_$TAG
timeout -k 10 900 python3 -u tools/ab_lib.py $R "$@" > gpurun_out/ab_$TAG/ab.log 2>&1 || exit $?
bash tools/sq_counters.sh $TAG
