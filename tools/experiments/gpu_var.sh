#!/bin/bash
# interleaved timing of library variants in separate processes: tools/gpu_var.sh ROUNDS base v1 v2 ...
set -o pipefail
R=$1; shift
for i in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = base ]; then V=""; else V=$v; fi
    OP_LIB_VARIANT=$V timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/var_${v}_$i.log 2>&1 || exit $?
  done
done
