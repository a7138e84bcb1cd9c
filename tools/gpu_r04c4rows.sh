#!/bin/bash
# Round 4: C4 second map-resize pass with row blocks (resize_cubic_f32_planar_mean_rows): the precise
# parity tests, then an interleaved A/B against the per-frame form (OP_CUBIC_ROWS=0) and G variants.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${AB_TAG:-r04c4rows}; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py tests/test_gpu_bench_configs.py -k "precise or Precise or cubic" > $O/tests.log 2>&1 || exit $?
AB_BENCH_ARGS="--precise --frame 720x1280 --steps 5 --warmup 1" timeout -k 10 900 python -u tools/ab_lib.py ${AB_ROUNDS:-3} ${AB_VARIANTS:-base OP_CUBIC_ROWS=0} > $O/ab.log 2>&1 || exit $?
echo done
