#!/bin/bash
# Round 4: Mconv6+7 fused heads with 4 tiles per workgroup (GEMM1 weights loaded once per 4 tiles;
# default, 3 workgroups per CU) vs one tile (OP_HEAD_TPW=1) vs 4 tiles at 2 workgroups per CU (occ2):
# headline A/B, then the parity files (bit-exact batch vs single frames covers both forms).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04t; mkdir -p $O
timeout -k 10 1100 python3 -u tools/ab_lib.py 4 base OP_HEAD_TPW=1 occ2 > $O/ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -m gpu > $O/tests.log 2>&1 || exit $?
echo done
