#!/bin/bash
# Bench lines: the default headline (side lines incl. batch-1 latency, CPU baseline unless
# NOCPU=1), C5-shaped 720p single scale and C4 multi-scale on 1280x720.   usage: tools/gpu_lines.sh TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/lines_$1; mkdir -p $O
X=""; [ -n "$NOCPU" ] && X="--no-cpu-baseline"
timeout -k 10 600 python -u bench.py $X > $O/default.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --frame 720x1280 > $O/c5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --precise --frame 720x1280 > $O/c4.log 2>&1 || exit $?
grep -h '^{' $O/*.log > $O/lines.jsonl
echo done
