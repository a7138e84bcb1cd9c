#!/bin/bash
set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "algos" > gpurun_out/m7_tests.log 2>&1 || exit $?
OP_HALO_MODE=7 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "forward or staged or detect" > gpurun_out/m7_tests2.log 2>&1 || exit $?
bash tools/gpu_exp.sh 7 42 m7 && bash tools/gpu_exp.sh 4 42 m4
