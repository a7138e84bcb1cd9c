#!/bin/bash
set -o pipefail
OP_HALO_MODE=4 OP_GRAPH_DRYRUN=1 timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/halo4.log 2>&1 || exit $?
for b in 42 28 84; do
  OP_HALO_MODE=4 timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --steps 10 > gpurun_out/b4_$b.log 2>&1 || exit $?
done
OP_HALO_MODE=3 timeout -k 10 200 python bench.py --batch 42 --no-cpu-baseline --steps 10 > gpurun_out/b3_42.log 2>&1 || exit $?
OP_HALO_MODE=4 bash tools/sq_counters.sh m4 --batch 42
