#!/bin/bash
# detect_precise side stream vs hardware queues: at 4 HW queues per process (HIP's default) the side
# stream shares a queue with the compute stream and nothing overlaps.  One-frame and 16-frame C4
# lines: no side stream / side stream at 8 queues / side stream at high priority with 4 queues;
# then the headline at 4 vs 8 queues.
set -o pipefail
OUT=gpurun_out/c4q; mkdir -p $OUT
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/$tag.log 2>&1 || return $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/$tag.log $tag | tee -a $OUT/summary.log
}
B1="--frame 720x1280 --precise --batch 1 --steps 10 --warmup 2"
C4="--frame 720x1280 --precise --steps 4 --warmup 1"
for r in 1 2; do
  line b1_q4_off_$r GPU_MAX_HW_QUEUES=4 OP_PRECISE_OVERLAP=0 -- $B1 || exit $?
  line b1_q8_on_$r GPU_MAX_HW_QUEUES=8 OP_PRECISE_OVERLAP=1 -- $B1 || exit $?
  line b1_q4_prio_$r GPU_MAX_HW_QUEUES=4 OP_PRECISE_OVERLAP=1 OP_SIDE_PRIORITY=1 -- $B1 || exit $?
done
line c4_q4_off GPU_MAX_HW_QUEUES=4 OP_PRECISE_OVERLAP=0 -- $C4 || exit $?
line c4_q8_on GPU_MAX_HW_QUEUES=8 OP_PRECISE_OVERLAP=1 -- $C4 || exit $?
line c4_q4_prio GPU_MAX_HW_QUEUES=4 OP_PRECISE_OVERLAP=1 OP_SIDE_PRIORITY=1 -- $C4 || exit $?
line head_q4 GPU_MAX_HW_QUEUES=4 -- --steps 20 || exit $?
line head_q8 GPU_MAX_HW_QUEUES=8 -- --steps 20 || exit $?
timeout -k 10 300 env GPU_MAX_HW_QUEUES=8 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_precise_full.py tests/test_gpu_parity.py -k "precise" > $OUT/tests_q8.log 2>&1 || exit $?
