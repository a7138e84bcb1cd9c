#!/bin/bash
# Round-3 profile of the default bench workload (kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes,
# tools/profile.sh) after the bench-configuration parity tests; with AB set, an interleaved A/B
# (tools/ab_lib.py) in the same call.   usage: [AB="base NAME=VAL"] tools/gpu_prof3.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out/ab_$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_configs.py \
  tests/test_gpu_forward_golden.py > gpurun_out/ab_$TAG/tests.log 2>&1 || exit $?
bash tools/profile.sh $TAG || exit $?
if [ -n "$AB" ]; then
  timeout -k 10 900 python3 -u tools/ab_lib.py ${ABR:-3} $AB > gpurun_out/ab_$TAG/ab.log 2>&1 || exit $?
fi
