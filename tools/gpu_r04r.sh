#!/bin/bash
# Round 4: LDS swizzle of conv_head's rows (noswz = off) and conv1_1's split stores as one
# ds_write_b128 per lane after a permlane16 row swap (c1noswap = off): headline A/B, one SQ pass,
# then the parity / bench-config files (bit-exact batch vs single frames, vs the oracle).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04r; mkdir -p $O
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base noswz c1noswap > $O/ab.log 2>&1 || exit $?
bash tools/sq_counters.sh r04r || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_configs.py tests/test_gpu_forward_golden.py -m gpu > $O/tests.log 2>&1 || exit $?
echo done
