#!/bin/bash
# Round 4: fused cubic map resize parity + C4 lines (fused / two-pass), then the batch-1 kernel trace.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04f; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_gpu_precise_full.py \
  tests/test_gpu_parity.py -k "precise or cubic" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --precise --frame 720x1280 > $O/c4.log 2>&1 || exit $?
OP_CUBIC_FUSED=0 timeout -k 10 300 python -u bench.py --precise --frame 720x1280 > $O/c4_twopass.log 2>&1 || exit $?
echo done
