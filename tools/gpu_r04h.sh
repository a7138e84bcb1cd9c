#!/bin/bash
# Round 4: whole GPU suite, C4 kernel trace, batch-1 A/B (joint 7x7 split), C5 A/B (4x48 tie rule).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 3 --warmup 1 --no-variants --no-profile > $O/c4prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_b1.sh r04h_joint "OP_M16_JOINT=1" "OP_M16_JOINT=0" 3 > $O/ab_joint.log 2>&1 || exit $?
for i in 1 2; do
  OP_M16K_TIE48=1 timeout -k 10 300 python -u bench.py --frame 720x1280 --no-cpu-baseline > $O/c5_tie_$i.log 2>&1 || exit $?
  OP_M16K_TIE48=0 timeout -k 10 300 python -u bench.py --frame 720x1280 --no-cpu-baseline > $O/c5_notie_$i.log 2>&1 || exit $?
done
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base w8 > $O/ab_w8.log 2>&1 || exit $?
echo done
