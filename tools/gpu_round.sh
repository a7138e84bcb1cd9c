#!/bin/bash
# Round evidence: GPU suite, default bench line, rocprofv3 stats + HBM PMC passes for the default workload.
set -o pipefail
TAG=${1:-r01}
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
bash tools/profile.sh $TAG || exit $?
