#!/bin/bash
# Round 4: conv_head hi/lo stores as one ds_write_b128 per lane (default) vs round 3's two 8-B
# stores (notswap): headline A/B + one SQ pass (LDS bank conflicts per kernel) on the product.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04q; mkdir -p $O
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base notswap > $O/ab_head_tswap.log 2>&1 || exit $?
bash tools/sq_counters.sh r04q || exit $?
echo done
