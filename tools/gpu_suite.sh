#!/bin/bash
# full GPU suite only
set -o pipefail
O=gpurun_out/suite; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
