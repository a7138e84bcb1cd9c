#!/bin/bash
# 7x7 tile-size selection: parity (auto + every forced NPX), batch sweep auto vs 640-px, C4, crops
set -o pipefail
O=gpurun_out/lat3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "forward or staged or precise or detect" > $O/tests.log 2>&1 || exit $?
for v in 8 6 5 3; do
  OP_M16_NPX=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "forward_368 or tile_sizes or forward_wide" > $O/tests_n$v.log 2>&1 || exit $?
done
for b in 1 4 8 16 24 38; do
  for v in 0 10; do
    OP_M16_NPX=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch $b > $O/b${b}_n$v.log 2>&1 || exit $?
  done
done
for v in 0 10; do
  OP_M16_NPX=$v timeout -k 10 300 python -u bench.py --precise --frame 720x1280 --batch 8 --steps 5 --warmup 1 > $O/c4_n$v.log 2>&1 || exit $?
  OP_M16_NPX=$v timeout -k 10 300 python -u bench.py --frame 720x1280 --batch 21 > $O/c5_n$v.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/bench_aux.py --no-cpu --only cpm > $O/aux.log 2>&1
