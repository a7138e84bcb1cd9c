#!/bin/bash
# Round 4: the joint 7x7 tile / split-K choice also costs the plain block order (one frame's
# Mconv1: 216 workgroups in one round instead of 288 XCD-padded slots): parity files, then the
# one-frame A/B vs HEAD (prev) and the batch-1 bench variant with its census.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_configs.py tests/test_gpu_cpm.py -m gpu > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab_b1.sh r04v_plain_small "OP_LIB_VARIANT=" "OP_LIB_VARIANT=prev" 3 > $O/ab_b1.log 2>&1 || exit $?
echo done
