#!/bin/bash
# 1) eager everywhere, per-kernel sync + guard bands  2) the real suite (graphs on) with guard bands
set -o pipefail
OP_GUARD=65536 OP_DEBUG_SYNC=1 OP_GRAPH_DRYRUN=1 timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/guard_eager.log 2>&1 || exit $?
OP_GUARD=65536 timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/guard_graph.log 2>&1 || exit $?
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/plain_graph.log 2>&1 || exit $?
