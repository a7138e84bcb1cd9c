#!/bin/bash
# Round 4: fused cubic parity + C4 kernel trace; batch-1 A/B of the joint 7x7 tile/split choice.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_uncapped.py tests/test_gpu_precise_full.py \
  > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "peaks or postprocess or staged or grouping or pose_detector" > $O/tests_post.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 3 --warmup 1 --no-variants --no-profile > $O/c4prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_b1.sh r04g_joint "OP_M16_JOINT=1" "OP_M16_JOINT=0" 3 > $O/ab_joint.log 2>&1 || exit $?
echo done
