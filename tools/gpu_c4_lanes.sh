#!/bin/bash
# (the OP_PRECISE_LANES switch lived only in the experiment build; the second lane was not kept)
# detect_precise: scale 1.5 on a second side stream (OP_PRECISE_LANES=2) vs one side stream (1):
# precise parity tests with two lanes, then interleaved one-frame and 16-frame C4 lines.
set -o pipefail
OUT=gpurun_out/lanes; mkdir -p $OUT
OP_PRECISE_LANES=2 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py -k "precise" > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log | tee -a $OUT/summary.log
for r in 1 2; do
  for v in 1 2; do
    OP_PRECISE_LANES=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b1_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('b1 lanes', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/b1_${v}_$r.log $v | tee -a $OUT/summary.log
    OP_PRECISE_LANES=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4 lanes', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/c4_${v}_$r.log $v | tee -a $OUT/summary.log
  done
done
