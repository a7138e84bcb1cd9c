#!/bin/bash
# Selected GPU test files (args), one pytest process, per-test timeout; log under gpurun_out/sel/
set -o pipefail
O=gpurun_out/sel; mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
