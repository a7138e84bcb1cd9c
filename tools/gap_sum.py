"""Idle time between kernels inside bench steps, from a rocprofv3 kernel-trace CSV.
A step starts at each conv1_pair launch; per step: wall span, busy (union of kernel intervals),
and the largest idle gaps with the kernels on either side.  gap_sum.py CSV [steps=3] [top=12]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
starts = [i for i, r in enumerate(rows) if "conv1_pair" in r["Kernel_Name"]]
sel = starts[-steps - 1:]  # the last `steps` whole steps (between consecutive step starts)
gaps = collections.Counter()
for a, b in zip(sel, sel[1:]):
    seg = rows[a:b]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    busy, end = 0, t0
    for i, r in enumerate(seg):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            prev = seg[i - 1]["Kernel_Name"][:48] if i else "-"
            gaps[(prev, r["Kernel_Name"][:48])] += s - end
        busy += max(0, e - max(s, end))
        end = max(end, e)
    print(f"step span {(t1 - t0) / 1e6:8.3f} ms  busy {busy / 1e6:8.3f} ms  idle {(t1 - t0 - busy) / 1e6:6.3f} ms  kernels {len(seg)}")
n = max(1, len(sel) - 1)
for (p, q), g in gaps.most_common(top):
    print(f"{g / n / 1e3:9.1f} us/step idle  after {p}  before {q}")
