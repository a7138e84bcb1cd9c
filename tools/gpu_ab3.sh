#!/bin/bash
# Parity of the bench configurations (incl. the kernels in use) + forward fixtures, then an
# interleaved A/B of env settings / library variants (tools/ab_lib.py).
# usage: tools/gpu_ab3.sh TAG ROUNDS spec...   (spec: base, a variant name, or NAME=VALUE[,NAME=VALUE])
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_configs.py \
  tests/test_gpu_forward_golden.py tests/test_gpu_cpm.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/ab_lib.py $R "$@" > $O/ab.log 2>&1
