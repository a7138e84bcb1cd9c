#!/bin/bash
# second SQ PMC pass (instruction mix) over a short bench run: tools/sq_counters2.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-sq}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/sq2_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS --kernel-trace --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile "$@" > $OUT/bench.log 2>&1
