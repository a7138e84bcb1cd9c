#!/bin/bash
set -o pipefail
OP_DEBUG_SYNC=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "cubic or precise" > gpurun_out/precise.log 2>&1 || exit $?
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
