#!/bin/bash
# C4 multi-scale: rocprofv3 kernel stats of bench.py --precise (1280x720, batch 8)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/precprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --batch 8 --steps 3 --warmup 1 --no-profile > $O/bench.log 2>&1
