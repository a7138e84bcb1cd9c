#!/bin/bash
# kernel-trace pass of the default bench workload for tools/gap_sum.py (GPU box, repo root)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/gaps; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-variants "$@" > $OUT/bench.log 2>&1 || exit $?
python3 $GRAFT_REPO_ROOT/tools/gap_sum.py $(ls $OUT/trace/*/*kernel_trace.csv $OUT/trace/*kernel_trace.csv 2>/dev/null | head -1) 4 16 > $OUT/gaps.txt
