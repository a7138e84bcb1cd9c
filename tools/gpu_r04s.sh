#!/bin/bash
# Round 4: 5-round interleaved headline A/B of the conv_head LDS swizzle (noswz = off) and the
# conv1_1 row-swapped b128 stores (c1noswap = off).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04s; mkdir -p $O
timeout -k 10 1100 python3 -u tools/ab_lib.py 5 base noswz c1noswap > $O/ab.log 2>&1 || exit $?
echo done
