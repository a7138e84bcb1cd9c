"""Per-kernel time per step from a rocprofv3 kernel-trace CSV: trace_sum.py CSV [steps] [top]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / steps:9.1f} us/step  n={len(v):4d}  {k}")
print(f"{sum(sum(v) for v in d.values()) / steps:9.1f} us/step total (incl. setup kernels)")
