set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 600 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_parity.py -k "gather or records or async or graph_replay or fetch_maps" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2c/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r2c/bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --precise --frame 720x1280 --batch 8 --steps 5 --warmup 2 > gpurun_out/r2c/bench_c4.log 2>&1
