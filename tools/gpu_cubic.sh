#!/bin/bash
set -o pipefail
O=gpurun_out/cubic; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "cubic or precise" > $O/tests.log 2>&1 || exit $?
bash tools/gpu_precise_prof.sh
