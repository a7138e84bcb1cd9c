#!/bin/bash
# GPU parity selection (forward / staged / graph / precise / CPM) + interleaved A/B of env settings.
# usage: tools/gpu_ab_env2.sh TAG ROUNDS spec...   (spec: base or NAME=VALUE[,NAME=VALUE])
set -o pipefail
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_forward_golden.py tests/test_gpu_parity.py tests/test_gpu_cpm.py -k "forward or staged or conv or graph or precise or cpm" > gpurun_out/$TAG/tests.log 2>&1 || exit $?
timeout -k 10 700 python3 -u tools/ab_lib.py $R "$@" > gpurun_out/$TAG/ab.log 2>&1
