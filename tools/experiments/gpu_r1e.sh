#!/bin/bash
set -o pipefail
OP_HALO_MODE=4 OP_GRAPH_DRYRUN=1 timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "forward or staged or detect" > gpurun_out/halo4.log 2>&1 || exit $?
OP_HALO_MODE=4 timeout -k 10 200 python bench.py --batch 42 --no-cpu-baseline --steps 10 > gpurun_out/exp_m4.log 2>&1 || exit $?
OP_HALO_MODE=5 timeout -k 10 200 python bench.py --batch 42 --no-cpu-baseline --steps 10 > gpurun_out/exp_m5.log 2>&1 || exit $?
OP_HALO_MODE=1 timeout -k 10 200 python bench.py --batch 28 --no-cpu-baseline --steps 10 > gpurun_out/exp_m1.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && mkdir -p $GRAFT_REPO_ROOT/gpurun_out/tr_m4 && OP_HALO_MODE=4 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_m4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --batch 42 > $GRAFT_REPO_ROOT/gpurun_out/tr_m4/bench.log 2>&1
