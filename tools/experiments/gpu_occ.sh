#!/bin/bash
set -o pipefail
O=gpurun_out/occ; mkdir -p $O
OP_M16_NPX=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "forward_368 or tile_sizes" > $O/tests_n3.log 2>&1 || exit $?
for b in 38 30 16; do
  for v in 10 3 2 0; do
    OP_M16_NPX=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch $b > $O/b${b}_n$v.log 2>&1 || exit $?
  done
done
