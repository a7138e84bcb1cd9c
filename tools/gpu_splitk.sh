#!/bin/bash
# 7x7 split-K for under-filled launches: full GPU suite, latency sweep (auto vs split off), crops
set -o pipefail
O=gpurun_out/splitk; mkdir -p $O
# (tests run separately)
for b in 1 4 8 38; do
  for v in 0 1; do
    OP_M16_KSPLIT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch $b > $O/b${b}_k$v.log 2>&1 || exit $?
  done
done
for v in 0 1; do
  OP_M16_KSPLIT=$v timeout -k 10 300 python -u bench.py --precise --frame 720x1280 --batch 8 --steps 5 --warmup 1 > $O/c4_k$v.log 2>&1 || exit $?
  OP_M16_KSPLIT=$v timeout -k 10 300 python -u tools/bench_aux.py --no-cpu --only cpm > $O/aux_k$v.log 2>&1 || exit $?
done
