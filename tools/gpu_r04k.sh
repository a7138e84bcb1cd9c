#!/bin/bash
# Round 4: fp32 fused head + in-kernel split-K (bit-exact tests), the parity file, a full bench
# line (headline + variants: fp32 classes, batch-1), the in-kernel split-K A/B on one frame, and
# the Winograd chunk micro-benchmark.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_forward_golden.py -m gpu > $O/parity.log 2>&1 || exit $?
timeout -k 10 600 python3 -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit $?
bash tools/gpu_ab_b1.sh r04k_inkernel "OP_SPLITK_INKERNEL=1" "OP_SPLITK_INKERNEL=0" 3 > $O/ab_inkernel.log 2>&1 || exit $?
timeout -k 10 120 tools/micro/l2_mfma_stream > $O/micro_4MiB.log 2>&1 || exit $?
timeout -k 10 120 tools/micro/l2_mfma_stream 16777216 > $O/micro_16MiB.log 2>&1 || exit $?
echo done
