"""Per-kernel mean FETCH_SIZE (raw KiB, no pattern factor) of one tools/gpu_fetch_ab.sh pass.
usage: python tools/fetch_sum.py gpurun_out/fetch_<tag>/<spec>"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(list)
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == "FETCH_SIZE":
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
print("==", os.path.basename(d.rstrip("/")))
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"  {k:60s} n={len(v):4d} mean={sum(v) / len(v) / 1024:9.1f} MiB total={sum(v) / 1024:10.1f} MiB")
