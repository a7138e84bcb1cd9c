set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05h; mkdir -p $O
OP_LIB_VARIANT=flags timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_configs.py tests/test_gpu_forward_golden.py tests/test_gpu_bench_default_mode.py -m gpu -k "not postprocess_bit_exact and not precise and not c4" > $O/flags_tests.log 2>&1 || exit $?
OP_LIB_VARIANT=stampsflags OP_M16_STAMPS=1 timeout -k 10 300 python -u bench.py --no-variants --no-cpu-baseline --steps 2 --warmup 1 --no-profile > $O/stamps_flags.log 2>&1 || exit $?
timeout -k 10 900 python3 -u tools/ab_lib.py 3 base flags nobar > $O/ab_flags.log 2>&1 || exit $?
echo done
