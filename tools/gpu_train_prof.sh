#!/bin/bash
# f4: training GPU tests, iteration time, rocprofv3 kernel stats
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/trainprof2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_aux.py --only train > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_aux.py --only train --iters 3 > $O/bench_prof.log 2>&1
