#!/bin/bash
set -o pipefail
OP_HALO_MODE=6 OP_GRAPH_DRYRUN=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "forward or staged or precise or detect" > gpurun_out/m6_tests.log 2>&1 || exit $?
OP_HALO_MODE=6 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp_m6.log 2>&1 || exit $?
OP_HALO_MODE=4 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp_m4.log 2>&1 || exit $?
