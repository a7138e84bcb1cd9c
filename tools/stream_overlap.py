"""Kernel-trace overlap between streams (rocprofv3 --kernel-trace --output-format csv).

  python tools/stream_overlap.py <kernel_trace.csv>

Per stream (or queue, when the trace has no stream id): kernel count and busy time; then, for every
pair of streams, the time during which both had a kernel running.  Answers whether work enqueued on
two HIP streams actually ran concurrently.
"""
import csv
import sys
from collections import defaultdict


def merge(iv):
    iv.sort()
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a = max(x[i][0], y[j][0])
        b = min(x[i][1], y[j][1])
        if b > a:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(path):
    rows = list(csv.DictReader(open(path)))
    key = "Stream_Id" if rows and "Stream_Id" in rows[0] else "Queue_Id"
    iv = defaultdict(list)
    names = defaultdict(lambda: defaultdict(int))
    for r in rows:
        s = r[key]
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        iv[s].append([a, b])
        names[s][r["Kernel_Name"].split("(")[0][:60]] += 1
    m = {s: merge(v) for s, v in iv.items()}
    for s in sorted(m):
        busy = sum(b - a for a, b in m[s])
        top = sorted(names[s].items(), key=lambda kv: -kv[1])[:3]
        print(f"{key} {s}: {len(iv[s])} kernels, busy {busy / 1e6:.3f} ms; top {top}")
    ss = sorted(m)
    for i in range(len(ss)):
        for j in range(i + 1, len(ss)):
            print(f"overlap {ss[i]} x {ss[j]}: {inter(m[ss[i]], m[ss[j]]) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
