#!/bin/bash
# Interleaved batch-size comparison of the default bench: tools/gpu_batch_ab.sh TAG ROUNDS B1 B2 ...
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for b in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-variants --batch $b --steps 10 --warmup 2 > $OUT/b${b}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['stage_ms_per_step'])" $OUT/b${b}_$r.log $r $b | tee -a $OUT/summary.log
  done
done
