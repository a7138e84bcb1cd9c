#!/bin/bash
# Per-kernel interleaved A/B of library variants by rocprofv3 kernel stats (GPU box, repo root):
#   tools/gpu_ab_kernel.sh ROUNDS PATTERN base v1 v2 ...  -> gpurun_out/ab_kernel/summary.log
# (base = the product library; vN = libopenpose_hip.vN.so via OP_LIB_VARIANT)
set -o pipefail
R=$1; PAT=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/ab_kernel; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in "$@"; do
    lib=$v; [ "$v" = base ] && lib=
    rm -rf $O/run_${v}_$r
    OP_LIB_VARIANT=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/run_${v}_$r -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-variants --no-profile > $O/run_${v}_$r.log 2>&1 || exit $?
    python3 - "$O/run_${v}_$r" "$PAT" "$v" "$r" <<'PY' | tee -a $O/summary.log
import csv, glob, json, sys
d, pat, v, r = sys.argv[1:5]
st = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = [x for x in csv.DictReader(open(st)) if pat in x["Name"]]
fps = [json.loads(l)["value"] for l in open(d + ".log") if l.startswith("{\"metric\"")][0]
print(r, v, fps, " ".join("%s=%.1fus" % (x["Name"].split("(")[0].replace("void ", "")[-40:], float(x["AverageNs"]) / 1e3) for x in rows))
PY
  done
done
