#!/bin/bash
# Round 3 (p): 64-channel x whole-tile 3x3 waves (OP_M16R_CBW=5) parity at the bench configurations,
# the whole GPU suite on the default tree, one bench line, then an interleaved A/B:
# vmw8 (the halo wait of the previous tree) / base / OP_M16R_CBW=5.
set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
OP_M16R_CBW=5 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_configs.py > $O/cbw5_bench_configs.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/ab_lib.py ${ABR:-3} vmw8 base OP_M16R_CBW=5 > $O/ab.log 2>&1 || exit $?
