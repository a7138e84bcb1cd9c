#!/bin/bash
# parity of the conv families + interleaved bench of halo modes: tools/gpu_algo.sh ROUNDS mode...
set -o pipefail
R=$1; shift
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "algos_agree or forward_368 or staged" > gpurun_out/algo_tests.log 2>&1 || exit $?
for i in $(seq 1 $R); do
  for m in "$@"; do
    OP_HALO_MODE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/alg_${m}_$i.log 2>&1 || exit $?
  done
done
