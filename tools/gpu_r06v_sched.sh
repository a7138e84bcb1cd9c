set -o pipefail
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_lib.py 3 base m16mx m16iinp m16iitr > $O/ab_headline.log 2>&1 &&
AB_BENCH_ARGS="--precise --frame 720x1280 --steps 5" timeout -k 10 400 python3 -u tools/ab_lib.py 3 base m16mx > $O/ab_c4.log 2>&1 &&
AB_BENCH_ARGS="--frame 720x1280" timeout -k 10 300 python3 -u tools/ab_lib.py 3 base m16mx > $O/ab_c5.log 2>&1 &&
AB_BENCH_ARGS="--batch 1 --steps 200 --warmup 20" timeout -k 10 300 python3 -u tools/ab_lib.py 3 base m16qii m16qmx > $O/ab_b1.log 2>&1
