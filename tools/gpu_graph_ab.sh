#!/bin/bash
# eager vs hipGraph-replay bench, interleaved on one box; graph-mode rocprofv3 stats for the 7x7 duration
set -o pipefail
TAG=${1:-gab}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "graph or staged_batch" > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --graph 0 > $O/eager_$i.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --no-cpu-baseline --graph 1 > $O/graph_$i.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --graph 1 > $GRAFT_REPO_ROOT/$O/stats_bench.log 2>&1
