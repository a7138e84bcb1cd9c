#!/bin/bash
# detect_precise small scales on the side stream: precise parity tests (overlap on, the default), then an
# interleaved A/B of the C4 bench line and of one-frame detect_precise, OP_PRECISE_OVERLAP=0 vs on.
set -o pipefail
OUT=gpurun_out/c4ov; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py -k "precise" > $OUT/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in 0 1; do
    OP_PRECISE_OVERLAP=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4 overlap', sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $OUT/c4_${v}_$r.log $v | tee -a $OUT/summary.log
  done
done
for v in 0 1; do
  OP_PRECISE_OVERLAP=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b1_${v}.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('b1 overlap', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/b1_${v}.log $v | tee -a $OUT/summary.log
done
