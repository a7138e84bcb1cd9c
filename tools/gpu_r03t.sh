#!/bin/bash
# Round 3 (t): the whole GPU suite, one bench line, and a kernel-trace profile of the bench on the
# random network's own maps (the dense post-process: sorted first-fit greedy, axis-tap tables).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r03t}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --maps network > $O/bench_net.log 2>&1 || exit $?
