#!/bin/bash
# C4 (multi-scale detect_precise, 1280x720): the precise parity tests, one C4 bench line and a
# kernel-trace profile of it.   usage: tools/gpu_c4.sh TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/c4_$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "precise or Precise or cubic" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --precise --frame 720x1280 > $O/c4.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --precise --frame 720x1280 --steps 3 --warmup 1 > $O/bench_prof.log 2>&1 || exit $?
