#!/bin/bash
# Round 4: the 7x7 kernel's first halo issued before the weight-ring prologue (first MFMAs wait for
# the halo and W(0), W(1) only) vs HEAD (prev): parity files, then one-frame and headline A/Bs.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_configs.py tests/test_gpu_forward_golden.py tests/test_gpu_precise_full.py -m gpu > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab_b1.sh r04u_prologue "OP_LIB_VARIANT=" "OP_LIB_VARIANT=prev" 3 > $O/ab_b1.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base prev > $O/ab_headline.log 2>&1 || exit $?
echo done
