#!/bin/bash
# Round 4: whole GPU suite; A/B product vs HEAD (conv1_pair ds_write_b128, XCD-local heat_fused);
# SQ counters of the C4 workload (fused cubic resize).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base prev > $O/ab_prev.log 2>&1 || exit $?
bash tools/sq_counters.sh r04j_c4 --precise --frame 720x1280 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $O/sq_insts -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 2 --warmup 1 --no-cpu-baseline --no-variants --no-profile > $O/sq_insts.log 2>&1 || exit $?
echo done
