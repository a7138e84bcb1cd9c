set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05k; mkdir -p $O
OP_F32_CB=4 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp32.py -m gpu > $O/cb4_tests.log 2>&1 || exit $?
AB_BENCH_ARGS="--precision fp32" timeout -k 10 900 python3 -u tools/ab_lib.py 2 OP_F32_CB=2 OP_F32_CB=4 > $O/ab_cb4.log 2>&1 || exit $?
echo done
