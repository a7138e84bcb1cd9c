#!/bin/bash
# f3/f4 rows: CPM GPU tests (incl. batched detect), then tools/bench_aux.py
set -o pipefail
O=gpurun_out/aux; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cpm.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_aux.py > $O/bench_aux.log 2>&1
