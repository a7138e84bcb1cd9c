#!/bin/bash
# graph dry-run dumps, then the co-split halo kernel (OP_HALO_MODE=3) through the GPU suite and bench
set -o pipefail
bash tools/graph_dbg.sh || exit $?
OP_HALO_MODE=3 OP_GRAPH_DRYRUN=1 timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/halo3.log 2>&1 || exit $?
for b in 21 28 42; do
  OP_HALO_MODE=3 timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --steps 10 > gpurun_out/b3_$b.log 2>&1 || exit $?
done
OP_HALO_MODE=1 timeout -k 10 200 python bench.py --batch 28 --no-cpu-baseline --steps 10 > gpurun_out/b1_28.log 2>&1 || exit $?
