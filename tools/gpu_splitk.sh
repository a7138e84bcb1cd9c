#!/bin/bash
# split-K (7x7 + 3x3) for under-filled launches: GPU suite, then latency A/B
set -o pipefail
O=gpurun_out/splitk2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for b in 1 2 4 38; do
  for v in 0 1; do
    OP_M16_KSPLIT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch $b > $O/b${b}_k$v.log 2>&1 || exit $?
  done
done
for v in 0 1; do
  OP_M16_KSPLIT=$v timeout -k 10 300 python -u bench.py --precise --frame 720x1280 --batch 8 --steps 5 --warmup 1 > $O/c4_k$v.log 2>&1 || exit $?
  OP_M16_KSPLIT=$v timeout -k 10 300 python -u tools/bench_aux.py --no-cpu --only cpm > $O/aux_k$v.log 2>&1 || exit $?
done
