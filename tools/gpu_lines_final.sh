#!/bin/bash
# Round-end lines with the package defaults (no env overrides): one-frame and 16-frame C4, C5-shaped
# single scale, then smoke + GPU suite + the default bench line (tools/gpu_final.sh).
set -o pipefail
OUT=gpurun_out/lines; mkdir -p $OUT
echo "GPU_MAX_HW_QUEUES in the box env: [${GPU_MAX_HW_QUEUES}]" > $OUT/summary.log
for a in "b1c4:--frame 720x1280 --precise --batch 1 --steps 10 --warmup 2" "c4:--frame 720x1280 --precise --steps 4 --warmup 1" "c5:--frame 720x1280 --steps 10 --warmup 2"; do
  tag=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/$tag.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" $OUT/$tag.log $tag | tee -a $OUT/summary.log
done
bash tools/gpu_final.sh
