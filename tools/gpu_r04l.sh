#!/bin/bash
# Round 4: split-K hand-off in sc1 form (no release fence): its bit-exact test, the gather tests
# (bounded keep slots), then the one-frame A/B in-kernel vs reduce launches.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_gather.py -m gpu > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab_b1.sh r04l_inkernel "OP_SPLITK_INKERNEL=1" "OP_SPLITK_INKERNEL=0" 3 > $O/ab_inkernel.log 2>&1 || exit $?
echo done
