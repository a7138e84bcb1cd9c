#!/bin/bash
# Round 4: grouping's per-connection block barriers as wave barriers (one-wave blocks, subsets in
# LDS; the HBM big mode keeps __syncthreads): post-process parity files, then A/Bs vs HEAD (prev) on
# the one-frame workload and the dense post-process line.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_uncapped.py tests/test_gpu_gather.py tests/test_gpu_precise_full.py -m gpu > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab_b1.sh r04z_wavebar "OP_LIB_VARIANT=" "OP_LIB_VARIANT=prev" 3 > $O/ab_b1.log 2>&1 || exit $?
for i in 1 2 3; do
  for v in "" prev; do
    OP_LIB_VARIANT=$v timeout -k 10 300 python bench.py --maps network --no-cpu-baseline --no-variants --steps 10 --warmup 2 > $O/net_${v:-base}_$i.log 2>&1 || exit $?
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/net_*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["stage_ms_per_step"].get("postprocess"))
PY
echo done
