#!/bin/bash
# The bench lines DESIGN.md quotes, one process each: the default headline (with its side lines and
# the CPU baseline), one-frame latency (eager, hipGraph replay), C5-shaped 720p single scale and C4
# multi-scale.   usage: tools/gpu_lines.sh TAG
set -o pipefail
O=gpurun_out/lines_$1; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/default.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --warmup 10 > $O/b1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --batch 1 --steps 50 --warmup 10 --graph 1 > $O/b1_graph.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --frame 720x1280 > $O/c5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --precise > $O/c4_368.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --precise --frame 720x1280 > $O/c4.log 2>&1 || exit $?
grep -h '^{' $O/*.log > $O/lines.jsonl
