#!/bin/bash
# Debug aid: capture the staged-path hipGraph without launching it (OP_GRAPH_DRYRUN) and dump it
# as DOT, once for the full GPU suite order and once for the isolated test.
set -o pipefail
mkdir -p gpurun_out/gfull gpurun_out/giso
OP_GRAPH_DRYRUN=1 OP_GRAPH_DUMP=gpurun_out/gfull timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gfull.log 2>&1 || exit $?
OP_GRAPH_DRYRUN=1 OP_GRAPH_DUMP=gpurun_out/giso timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -k staged_batch -x -q > gpurun_out/giso.log 2>&1 || exit $?
