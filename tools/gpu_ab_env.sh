#!/bin/bash
# A/B of an env knob on the default bench, interleaved: tools/gpu_ab_env.sh <tag> "<ENV=a>" "<ENV=b>" [rounds]
set -o pipefail
TAG=$1; A=$2; B=$3; N=${4:-2}
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  env $A timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $OUT/a_$i.log 2>&1 || exit $?
  env $B timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $OUT/b_$i.log 2>&1 || exit $?
done
python - "$OUT" <<'PY'
import json, sys, glob
for side in "ab":
    vals = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob(sys.argv[1] + "/%s_*.log" % side))]
    print(side, vals)
PY
