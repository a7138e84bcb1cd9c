#!/bin/bash
# Round 4: 7x7 tile sizes NPX 9 / 7 in the cost model's candidates: the full GPU suite, then
# interleaved A/Bs against OP_M16_ODD=0 on the headline, and of OP_M16_ODD_SPLIT=1 on one frame.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04odd; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/ab_lib.py 3 base OP_M16_ODD=0 > $O/ab_headline.log 2>&1 || exit $?
bash tools/gpu_ab_b1.sh r04odd_b1 "OP_M16_ODD_SPLIT=0" "OP_M16_ODD_SPLIT=1" 3 > $O/ab_b1.log 2>&1 || exit $?
echo done
