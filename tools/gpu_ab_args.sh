#!/bin/bash
# Interleaved A/B of bench.py argument sets on one box (GPU box, repo root):
#   tools/gpu_ab_args.sh ROUNDS "args A" "args B" ...   -> gpurun_out/ab_args/summary.log
set -o pipefail
O=gpurun_out/ab_args; mkdir -p $O
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --steps 20 --warmup 3 $a > $O/v${i}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], repr(sys.argv[3]), d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))" $O/v${i}_$r.log $r "$a" | tee -a $O/summary.log
  done
done
