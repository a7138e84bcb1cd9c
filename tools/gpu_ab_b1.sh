#!/bin/bash
# Interleaved A/B of an env knob on the one-frame workload (bench.py --batch 1):
#   tools/gpu_ab_b1.sh <tag> "<ENV=a>" "<ENV=b>" [rounds]
set -o pipefail
TAG=$1; A=$2; B=$3; N=${4:-3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab_$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  env $A timeout -k 10 200 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-variants > $OUT/a_$i.log 2>&1 || exit $?
  env $B timeout -k 10 200 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-variants > $OUT/b_$i.log 2>&1 || exit $?
done
python - "$OUT" <<'PY'
import json, sys, glob
for side in "ab":
    for f in sorted(glob.glob(sys.argv[1] + "/%s_*.log" % side)):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(side, d["value"], d["ms_per_step"], d["stage_ms_per_step"])
PY
