#!/bin/bash
# C4 parity tests, then an interleaved A/B of the C4 bench line: product library vs OP_LIB_VARIANT=$1.
set -o pipefail
V=${1:-prev}
OUT=gpurun_out/c4ab; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py -k "precise" > $OUT/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in base $V; do
    OP_LIB_VARIANT=$([ $v = base ] && echo "" || echo $v) timeout -k 10 300 python bench.py --frame 720x1280 --precise --steps 4 --warmup 1 > $OUT/${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $OUT/${v}_$r.log $v | tee -a $OUT/summary.log
  done
done
