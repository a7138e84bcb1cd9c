#!/bin/bash
# Single-frame (batch 1) latency vs the 7x7 tile size (OP_M16_NPX) and split-K factor (OP_M16_KSPLIT).
set -o pipefail
OUT=gpurun_out/b1sweep; mkdir -p $OUT
for npx in 0 2 4 5 8 10; do
  for ks in 0 2 4 8; do
    OP_M16_NPX=$npx OP_M16_KSPLIT=$ks timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --batch 1 --steps 50 --warmup 5 > $OUT/n${npx}_k${ks}.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('npx', sys.argv[2], 'ks', sys.argv[3], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $OUT/n${npx}_k${ks}.log $npx $ks | tee -a $OUT/summary.log
  done
done
