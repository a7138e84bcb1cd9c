#!/bin/bash
# Deep weight ring for small 7x7 tiles: parity selection, then batch 1/2/4/8 latency with and without it.
set -o pipefail
OUT=gpurun_out/b1deep; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_forward_golden.py tests/test_gpu_parity.py tests/test_gpu_cpm.py -k "forward or staged or conv or graph or precise or cpm or tile" > $OUT/tests.log 2>&1 || exit $?
for r in 1 2; do
  for b in 1 2 4 8 16; do
    for nd in 0 1; do
      OP_M16_NODEEP=$nd timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --batch $b --steps 30 --warmup 5 > $OUT/b${b}_nd${nd}_$r.log 2>&1 || exit $?
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('batch', sys.argv[2], 'nodeep', sys.argv[3], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $OUT/b${b}_nd${nd}_$r.log $b $nd | tee -a $OUT/summary.log
    done
  done
done
