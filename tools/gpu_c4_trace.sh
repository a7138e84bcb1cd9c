#!/bin/bash
# Kernel trace of one-frame detect_precise (4 scales) with the side stream, and the per-stream
# busy / overlap summary (tools/stream_overlap.py).  GPU_MAX_HW_QUEUES=8 is what the loader sets;
# it is exported here too because the profiler's preloaded library may start HIP first.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c4trace; mkdir -p $OUT
GPU_MAX_HW_QUEUES=8 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o b1 -- python3 bench.py --frame 720x1280 --precise --batch 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b1.log 2>&1 || exit $?
f=$(find $OUT/raw -name '*kernel_trace.csv' | head -n 1)
python tools/stream_overlap.py "$f" > $OUT/overlap.txt 2>&1
cat $OUT/overlap.txt
