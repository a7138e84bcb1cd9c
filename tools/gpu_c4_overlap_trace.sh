#!/bin/bash
# Does the detect_precise side stream overlap the large scales?  Kernel trace of one-frame and
# 16-frame C4 runs (start/end per kernel, queue and stream ids), then the one-frame A/B again with
# more hardware queues per process.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/c4tr; mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/b1 -o b1 -- python3 bench.py --frame 720x1280 --precise --batch 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b1_trace.log 2>&1 || exit $?
for q in 4 8; do
  for v in 0 1; do
    GPU_MAX_HW_QUEUES=$q OP_PRECISE_OVERLAP=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b1_q${q}_${v}.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('b1 queues', sys.argv[2], 'overlap', sys.argv[3], d['value'], d['ms_per_step'])" $OUT/b1_q${q}_${v}.log $q $v | tee -a $OUT/summary.log
  done
done
