#!/bin/bash
set -o pipefail
O=gpurun_out/bsweep2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "forward or staged or detect" > $O/tests.log 2>&1 || exit $?
for b in 38 40 48 57 76 1 16; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --batch $b > $O/b$b.log 2>&1 || exit $?
done
