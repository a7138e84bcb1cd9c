#!/bin/bash
# Round 4: kernel trace of the one-frame workload (bench.py --batch 1), per-kernel time per frame and
# the idle gaps between kernels.   usage: tools/gpu_r04b1trace.sh TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/b1trace_$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --batch 1 --steps 40 --warmup 10 --no-cpu-baseline --no-variants --no-profile > $O/bench.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/trace_sum.py $O/tr/run_kernel_trace.csv 50 30 > $O/trace_sum.txt || exit $?
python3 tools/gap_sum.py $O/tr/run_kernel_trace.csv 5 20 > $O/gap_sum.txt || exit $?
echo done
