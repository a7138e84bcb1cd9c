#!/bin/bash
# batch sweep + rocprofv3 kernel stats (run on the GPU box from the repo root)
set -o pipefail
mkdir -p gpurun_out
for b in 8 15 16 31 32; do
  timeout -k 10 240 python bench.py --steps 6 --warmup 2 --batch $b --no-cpu-baseline > gpurun_out/sweep_b$b.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --batch 16 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --batch 16 --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --batch 16 --no-cpu-baseline --no-profile > $GRAFT_REPO_ROOT/gpurun_out/pmc_write.log 2>&1 || exit $?
