"""Per-launch durations of one bench step from a rocprofv3 kernel trace, with algorithmic TF/s for
the conv launches (layer order of the staged forward).  usage: layer_times.py <trace.csv> <batch>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
B = int(sys.argv[2])
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# one step starts at the preprocess kernel; take the last complete step
starts = [i for i, r in enumerate(rows) if any(k in r["Kernel_Name"] for k in ("preprocess", "conv11", "conv1_pair"))]
i0 = starts[-2] if len(starts) > 1 else starts[0]
i1 = starts[-1] if len(starts) > 1 else len(rows)
# logical conv FLOPs per frame, in launch order of the split plan (368x368)
def f(ci, co, k, h):
    return 2.0 * ci * co * k * k * h * h
fused1 = any("conv1_pair" in r["Kernel_Name"] for r in rows[i0:i1])
head = any("conv_head" in r["Kernel_Name"] for r in rows[i0:i1])
plan = ([f(3, 64, 3, 368) + f(64, 64, 3, 368)] if fused1 else [f(3, 64, 3, 368), f(64, 64, 3, 368)])
plan += [f(64, 128, 3, 184), f(128, 128, 3, 184),
         f(128, 256, 3, 92), f(256, 256, 3, 92), f(256, 256, 3, 92), f(256, 256, 3, 92),
         f(256, 512, 3, 46), f(512, 512, 3, 46), f(512, 256, 3, 46), f(256, 128, 3, 46),
         f(128, 256, 3, 46), 2 * f(128, 128, 3, 46), 2 * f(128, 128, 3, 46)]
h1 = [2 * f(128, 512, 1, 46) + f(512, 38, 1, 46) + f(512, 19, 1, 46)]
plan += h1 if head else [2 * f(128, 512, 1, 46), f(512, 38, 1, 46) + f(512, 19, 1, 46)]
for s_ in range(5):
    plan += [f(185, 256, 7, 46)] + [2 * f(128, 128, 7, 46)] * 4
    h = [2 * f(128, 128, 1, 46) + f(128, 38, 1, 46) + f(128, 19, 1, 46)]
    plan += h if head else [2 * f(128, 128, 1, 46), f(128, 38, 1, 46) + f(128, 19, 1, 46)]
j = 0
tot = 0.0
for r in rows[i0:i1]:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    tot += dt
    fl = ""
    if "conv" in name:
        if j < len(plan):
            p = plan[j]
            j += 1
            if p:
                fl = "%7.1f TF/s" % (p * B / (dt * 1e-3) / 1e12)
    print("%-55s %8.3f ms %s" % (name[:55], dt, fl))
print("total %.3f ms" % tot)
