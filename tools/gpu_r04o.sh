#!/bin/bash
# Round 4: split-K reduce kernels with all partials loaded before the first add -- one-frame A/B
# vs HEAD's library (prev), then the split-K parity tests on the product library.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04o; mkdir -p $O
bash tools/gpu_ab_b1.sh r04o_reduce_unroll "OP_LIB_VARIANT=" "OP_LIB_VARIANT=prev" 3 > $O/ab_b1.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "splitk or tile_sizes or staged" -m gpu > $O/tests.log 2>&1 || exit $?
echo done
