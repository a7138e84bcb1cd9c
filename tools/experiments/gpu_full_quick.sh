#!/bin/bash
# full GPU suite, then the default bench and one traced bench (per-layer times)
set -o pipefail
TAG=${1:-q}
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp_$TAG.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && mkdir -p $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/tr_$TAG/bench.log 2>&1
