#!/bin/bash
# Round 3: the new parity tests first (verbose), then the whole GPU suite, then one bench line.
set -o pipefail
O=gpurun_out/r03check; mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_configs.py tests/test_gpu_gather.py tests/test_gpu_train.py \
  tests/test_gpu_parity.py -k "bench or gather or train or precise_mode or cli_on_person" > $O/new_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
if [ -n "$AB" ]; then
  timeout -k 10 900 python3 -u tools/ab_lib.py ${ABR:-3} $AB > $O/ab.log 2>&1 || exit $?
fi
