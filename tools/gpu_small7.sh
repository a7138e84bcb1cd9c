#!/bin/bash
# small-launch 7x7 tiles: full GPU suite, aux bench (single-crop latency), default bench
set -o pipefail
O=gpurun_out/small7; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_aux.py --no-cpu --only cpm > $O/aux_small.log 2>&1 || exit $?
OP_M16_SMALL=0 timeout -k 10 300 python -u tools/bench_aux.py --no-cpu --only cpm > $O/aux_big.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
