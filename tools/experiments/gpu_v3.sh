#!/bin/bash
set -o pipefail
for v in 1 2; do
OP_BIG3=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "forward_368 or staged_batch" > gpurun_out/v3_$v.log 2>&1 || exit $?
done
for v in 0 1 2; do
OP_BIG3=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp_v3_$v.log 2>&1 || exit $?
done
