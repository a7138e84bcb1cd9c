#!/bin/bash
set -o pipefail
OP_HALO_MODE=4 OP_GRAPH_DRYRUN=1 timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "forward or staged" > gpurun_out/halo4.log 2>&1 || exit $?
OP_HALO_MODE=4 timeout -k 10 200 python bench.py --batch 42 --no-cpu-baseline --steps 10 > gpurun_out/b4_42.log 2>&1 || exit $?
OP_BIG_PLAIN_ORDER=1 OP_HALO_MODE=4 timeout -k 10 200 python bench.py --batch 42 --no-cpu-baseline --steps 10 > gpurun_out/b4p_42.log 2>&1 || exit $?
