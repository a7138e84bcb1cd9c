#!/bin/bash
# Round 4: L2-stream micro (Winograd costing); fused cubic (G 2) parity + C4 trace; batch-1 trace;
# C4 line; Mconv1 pair-major A/B.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04i; mkdir -p $O
timeout -k 10 120 tools/micro/l2_mfma_stream > $O/l2_mfma_stream_4MiB.log 2>&1 || exit $?
timeout -k 10 120 tools/micro/l2_mfma_stream 16777216 > $O/l2_mfma_stream_16MiB.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_precise_full.py > $O/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 3 --warmup 1 --no-variants --no-profile > $O/c4prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b1prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 1 --steps 40 --warmup 5 --no-cpu-baseline --no-variants --no-profile > $O/b1prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --precise --frame 720x1280 > $O/c4.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/ab_lib.py 3 OP_M16_PAIR=1 OP_M16_PAIR=0 > $O/ab_pair.log 2>&1 || exit $?
echo done
