#!/bin/bash
# Round 4: the split-K cost term of the joint 7x7 tile / split choice (OP_M16_SPLIT_GAMMA, default
# 0.2 of a chunk-step per split) on the one-frame workload.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r04w; mkdir -p $O
for i in 1 2 3; do
  for g in 0.2 0.05 0.5 1.0; do
    OP_M16_SPLIT_GAMMA=$g timeout -k 10 200 python bench.py --batch 1 --steps 200 --warmup 20 --no-cpu-baseline --no-variants > $O/g${g}_$i.log 2>&1 || exit $?
  done
done
python - "$O" <<'PY'
import json, sys, glob, statistics
res = {}
for f in sorted(glob.glob(sys.argv[1] + "/g*.log")):
    g = f.split("/")[-1][1:].rsplit("_", 1)[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    res.setdefault(g, []).append((d["ms_per_step"], d["stage_ms_per_step"]["conv7x7"]))
for g, v in res.items():
    print("gamma", g, "ms/frame median", statistics.median(x[0] for x in v), "conv7x7", statistics.median(x[1] for x in v))
PY
