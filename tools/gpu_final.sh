#!/bin/bash
# round-end check: smoke(), full GPU suite, default bench line
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
