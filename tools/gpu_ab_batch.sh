#!/bin/bash
# conv-family parity tests, then interleaved bench runs of "mode:batch" pairs: tools/gpu_ab_batch.sh ROUNDS 4:42 9:46 ...
set -o pipefail
R=$1; shift
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "algos_agree or forward_368 or staged" > gpurun_out/algo_tests.log 2>&1 || exit $?
for i in $(seq 1 $R); do
  for mb in "$@"; do
    m=${mb%%:*}; b=${mb##*:}
    OP_HALO_MODE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --batch $b > gpurun_out/abb_${m}_${b}_$i.log 2>&1 || exit $?
  done
done
