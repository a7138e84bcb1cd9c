#!/bin/bash
# The non-headline bench lines on the current build (GPU box, repo root): C4 multi-scale 1280x720,
# C5-shaped 1280x720 single scale, single-frame latency (eager and hipGraph).
set -o pipefail
O=gpurun_out/lines; mkdir -p $O
timeout -k 10 300 python bench.py --precise --frame 720x1280 --steps 5 --warmup 2 > $O/c4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --frame 720x1280 --steps 10 --warmup 3 > $O/c5.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-variants > $O/b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-variants --graph 1 > $O/b1_graph.log 2>&1 || exit $?
for f in c4 c5 b1 b1_graph; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), d['config']['frames_per_step_per_gpu'], d.get('persons_per_s'))" $O/$f.log $f | tee -a $O/summary.log
done
