#!/bin/bash
# Round-end: rocprofv3 kernel stats of the C4 line (16 frames, small scales on the side stream), then
# smoke + GPU suite + the default bench line (tools/gpu_final.sh).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/c4end; mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --frame 720x1280 --precise --steps 3 --warmup 1 --no-profile --no-cpu-baseline > $OUT/prof_c4.log 2>&1) || exit $?
f=$(find $OUT/stats -name '*kernel_stats.csv' | head -n 1); cp "$f" $OUT/kernel_stats.csv
t=$(find $OUT/stats -name '*kernel_trace.csv' | head -n 1); python tools/stream_overlap.py "$t" > $OUT/overlap.txt 2>&1
rm -rf $OUT/stats
bash tools/gpu_final.sh
