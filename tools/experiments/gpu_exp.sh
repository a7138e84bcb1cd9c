#!/bin/bash
# bench each experiment variant of the library: tools/gpu_exp.sh <mode> <batch> <variant...>
set -o pipefail
MODE=$1; B=$2; shift 2
for v in "$@"; do
  if [ "$v" = base ]; then V=""; else V=$v; fi
  OP_LIB_VARIANT=$V OP_HALO_MODE=$MODE timeout -k 10 200 python bench.py --batch $B --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/exp_$v.log 2>&1 || exit $?
done
