"""Idle time between kernels in one bench step from a rocprofv3 kernel-trace CSV:
gaps.py <trace.csv> [top]  -- step span vs summed kernel time, and the largest gaps (with the
kernel after each)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "conv11" in r["Kernel_Name"] or "conv1_pair" in r["Kernel_Name"]]
i0, i1 = starts[-2], starts[-1]
step = rows[i0:i1]
span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step) / 1e3
gaps = []
for a, b in zip(step, step[1:]):
    gaps.append(((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3, b["Kernel_Name"][:60]))
print("kernels %d  span %.1f us  busy %.1f us  idle %.1f us (%.1f %%)  next-step gap %.1f us"
      % (len(step), span, busy, span - busy, 100 * (span - busy) / span,
         (int(rows[i1]["Start_Timestamp"]) - int(step[-1]["End_Timestamp"])) / 1e3))
for g, k in sorted(gaps, reverse=True)[:top]:
    print("%8.1f us before %s" % (g, k))
