#!/bin/bash
# preprocess_cubic with host-computed scales vs the HEAD library (OP_LIB_VARIANT=head, tools/build_rev.sh):
# averaged detect_precise maps bit-identical, precise parity tests, C4 / one-frame A/B.
set -o pipefail
OUT=gpurun_out/prepab; mkdir -p $OUT
timeout -k 10 200 python tools/cubic_ab_maps.py $OUT/new.npz > $OUT/maps.log 2>&1 || exit $?
OP_LIB_VARIANT=head timeout -k 10 200 python tools/cubic_ab_maps.py $OUT/old.npz >> $OUT/maps.log 2>&1 || exit $?
python tools/cubic_ab_maps.py --compare $OUT/new.npz $OUT/old.npz | tee -a $OUT/summary.log || exit $?
rm -f $OUT/*.npz
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py -k "precise or cubic" > $OUT/tests.log 2>&1 || exit $?
tail -1 $OUT/tests.log | tee -a $OUT/summary.log
for r in 1 2; do
  for v in head new; do
    OP_LIB_VARIANT=$([ $v = new ] && echo "" || echo $v) timeout -k 10 300 python bench.py --frame 720x1280 --precise --batch 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b1_${v}_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('b1', sys.argv[2], d['value'], d['ms_per_step'])" $OUT/b1_${v}_$r.log $v | tee -a $OUT/summary.log
  done
done
