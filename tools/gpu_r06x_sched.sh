# The post-RA-off flags for conv_m16 / conv_m16r (product library) against the previous product
# (prev): bench-config parity first, then headline / C4 A/Bs; conv1_pair under iterative-ilp with
# post-RA off (c1pii, built on prev's flags), the fp32 line with conv_f32's post-RA off (f32nopost),
# post-RA off for the small-launch 3x3 objects (np3) and for the heads / heat / one-frame 7x7 (nphd).
set -o pipefail
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_configs.py \
  tests/test_gpu_forward_golden.py > $O/tests.log 2>&1 &&
timeout -k 10 500 python3 -u tools/ab_lib.py 4 prev base c1pii np3 nphd > $O/ab_headline.log 2>&1 &&
AB_BENCH_ARGS="--precision fp32 --no-side-lines --steps 4" timeout -k 10 400 python3 -u tools/ab_lib.py 3 prev f32nopost > $O/ab_fp32.log 2>&1 &&
AB_BENCH_ARGS="--precise --frame 720x1280 --steps 5" timeout -k 10 400 python3 -u tools/ab_lib.py 3 prev base > $O/ab_c4.log 2>&1 &&
AB_BENCH_ARGS="--batch 1 --steps 200 --warmup 20" timeout -k 10 300 python3 -u tools/ab_lib.py 3 base np3 nphd > $O/ab_b1.log 2>&1
