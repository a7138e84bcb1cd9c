#!/bin/bash
# (the OP_CUBIC_FLAT switch lived only in the experiment build; the kernel was not kept)
# First map resize of detect_precise: 3D-grid kernel vs the flat-index form (OP_CUBIC_FLAT=1):
# maps bit-identical, precise parity tests, then an interleaved A/B of the C4 and one-frame lines.
set -o pipefail
OUT=gpurun_out/cubab; mkdir -p $OUT
timeout -k 10 200 python tools/cubic_ab_maps.py $OUT/new.npz > $OUT/maps.log 2>&1 || exit $?
OP_CUBIC_FLAT=1 timeout -k 10 200 python tools/cubic_ab_maps.py $OUT/old.npz >> $OUT/maps.log 2>&1 || exit $?
python tools/cubic_ab_maps.py --compare $OUT/new.npz $OUT/old.npz | tee -a $OUT/summary.log || exit $?
rm -f $OUT/*.npz
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py -k "precise or cubic" > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log | tee -a $OUT/summary.log
for r in 1 2; do
  for v in 1 0; do
    OP_CUBIC_FLAT=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --steps 4 --warmup 1 --no-cpu-baseline > $OUT/c4_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4 flat', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/c4_${v}_$r.log $v | tee -a $OUT/summary.log
    OP_CUBIC_FLAT=$v timeout -k 10 300 python bench.py --frame 720x1280 --precise --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b1_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('b1 flat', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/b1_${v}_$r.log $v | tee -a $OUT/summary.log
  done
done
