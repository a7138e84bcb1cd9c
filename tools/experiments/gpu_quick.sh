#!/bin/bash
# quick perf check: forward/staged GPU parity subset, default bench, one traced bench for per-layer times
set -o pipefail
TAG=${1:-q}
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "forward or staged or precise" > gpurun_out/quick_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp_$TAG.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && mkdir -p $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG/bench.log 2>&1
