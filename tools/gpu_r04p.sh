#!/bin/bash
# Round 4: fused-head workgroups of 128 px on large launches (default) vs 64 px, headline A/B;
# then the bench-config parity file (bit-exact batch vs single frames covers both head sizes).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04p; mkdir -p $O
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base OP_HEAD_PX=64 > $O/ab_head_px.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_configs.py -m gpu > $O/tests.log 2>&1 || exit $?
echo done
